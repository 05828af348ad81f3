"""GPU: device-resident searches issued on several streams at once (up to WS_MAX = 4
scratch sets per index, csrc/vsg_index.cpp ws_acquire) return exactly what the same
searches return one after another -- HNSW, filtered (tombstones) and exact."""
import numpy as np
import pytest
import torch

import vsg
from vsg import datagen as G

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["hnsw", "filtered", "exact"])
def test_concurrent_streams_equal_sequential(mode):
    n, dim, nq = 30000, 64, 3000
    bs, qs, ms = G.config_seeds(1)
    x = G.clustered(n, dim, bs, ms)
    idx = vsg.Index(dim, "l2sq", "f32", 16, 128, 64, seed=4)
    idx.add(np.arange(n), x)
    if mode == "filtered":
        idx.remove(np.arange(0, n, 3))
    qa = torch.from_numpy(G.clustered(5 * nq, dim, qs, ms)).cuda()
    batches = [qa[i * nq:(i + 1) * nq].contiguous() for i in range(5)]
    exact = mode == "exact"
    ref = []
    for b in batches:
        k, d = idx.search_device(b, 10, 48, exact=exact)
        torch.cuda.synchronize()
        ref.append((k.clone(), d.clone()))
    streams = [torch.cuda.Stream() for _ in range(3)]
    for _ in range(3):  # rounds: workspaces reused across streams
        outs = []
        for i, b in enumerate(batches):
            s = streams[i % 3]
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                k = torch.empty((nq, 10), dtype=torch.int64, device="cuda")
                d = torch.empty((nq, 10), dtype=torch.float32, device="cuda")
                idx.search_device(b, 10, 48, out_keys=k, out_dist=d, stream=s.cuda_stream, exact=exact)
            outs.append((k, d))
        torch.cuda.synchronize()
        for (k, d), (rk, rd) in zip(outs, ref):
            assert torch.equal(k, rk) and torch.equal(d, rd)
