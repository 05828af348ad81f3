"""Parity at the C4 configuration (BASELINE.json configs[3]): 128-d SIFT-like
integer data (clustered latent, ReLU, x48, rounded into 0..255), f16 HBM storage, L2sq,
M=16, efC=128; the full config is 100M rows as 8 row shards of 12.5M (VERDICT r2 missing
#2 / next #1).  Reference call sites: usearch::Index::add and search,
/root/reference/src/index/usearch.rs:221, 275-277.

The data is integer-valued, so every f16 element is exact and every squared L2 sum is an
integer below 128 * 255^2 < 2^24: exact in f32 whatever the summation order.  That makes
the 16-chunk f16 kernel instances comparable with the oracle (f32 rows) bit for bit:
  (a) oracle-built 20k-row graph (with tombstones) imported into an f16 index: GPU search
      == oracle search, keys and distances, at ef 64 / 192 / 1024 (the register kernel's
      R classes up to its largest);
  (b) GPU-built 200k-row graph: recall@10 within +-0.5 % of the oracle's own build at
      ef 64 and 192, same ground truth (two-sided: a GPU graph much better than the
      restatement's would be a divergence too);
  (c) one full C4 shard, 12.5M x 128 f16 built on the GPU: recall@10 >= 0.95 at ef 192 on
      10,000 queries against the GPU exact search, and that exact search checked against
      numpy on 1,000 queries -- bit for bit, since the distances are exact integers and
      ties break by (distance, row) on both sides.
"""
import numpy as np
import pytest

import oracle as O
import vsg
from vsg import datagen as G

pytestmark = [pytest.mark.gpu]

DIM, M, EFC, K = 128, 16, 128, 10
BS, QS, MS = G.config_seeds(3)  # C4 seed set


def recall(found, truth, k=K):
    return float(np.mean([len(set(found[i][:k].tolist()) & set(truth[i][:k].tolist())) / k
                          for i in range(truth.shape[0])]))


def _cores():
    from bench import host_cores
    return host_cores()


@pytest.mark.timeout(300)
def test_c4_f16_search_on_oracle_graph_bitexact():
    n, nq = 20000, 300
    x = G.sift_like(n, DIM, BS, MS)
    q = G.sift_like(nq, DIM, QS, MS)
    assert np.all(x == np.rint(x)) and x.max() <= 255 and x.min() >= 0
    h = O.HnswOracle(DIM, "l2sq", M, EFC, 64, seed=17)
    h.add(np.arange(n), x, threads=_cores())
    h.remove(np.arange(0, n, 31))
    idx = vsg.Index(DIM, "l2sq", "f16", M, EFC, 64, seed=17)
    idx.import_graph(h.export())
    assert idx.size() == h.size()
    for ef in (64, 192, 1024):
        for k in (K, 100):
            ok, od, oc = h.search(q, k, ef, threads=_cores())
            m = idx.search(q, k, ef)
            np.testing.assert_array_equal(m.counts, oc)
            np.testing.assert_array_equal(m.keys, ok, err_msg=f"ef {ef} k {k}")
            np.testing.assert_array_equal(m.distances, od, err_msg=f"ef {ef} k {k}")


@pytest.mark.timeout(600)
def test_c4_gpu_build_recall_vs_oracle_build():
    n, nq = 200_000, 5000
    x = G.sift_like(n, DIM, BS, MS)
    q = G.sift_like(nq, DIM, QS, MS)
    gpu = vsg.Index(DIM, "l2sq", "f16", M, EFC, 64, seed=0x5EED)
    gpu.add(np.arange(n), x)
    gt = gpu.exact_search(q, K)
    # the f16 VALU exact kernel is the ground truth: bit-exact vs the oracle on a subset
    ok, od, _ = O.exact_search("l2sq", x, q[:300], K, threads=_cores())
    np.testing.assert_array_equal(gt.keys[:300], ok)
    np.testing.assert_array_equal(gt.distances[:300], od)
    O.set_fast_metric(True)
    try:
        orc = O.HnswOracle(DIM, "l2sq", M, EFC, 64, seed=0x5EED)
        orc.add(np.arange(n), x, threads=_cores())
        for ef in (64, 192):
            rc = recall(orc.search(q, K, ef, threads=_cores())[0], gt.keys)
            rg = recall(gpu.search(q, K, ef).keys, gt.keys)
            print(f"C4 200k ef={ef}: GPU build {rg:.4f}, oracle build {rc:.4f}")
            assert abs(rg - rc) <= 0.005, (ef, rg, rc)
    finally:
        O.set_fast_metric(False)


def _numpy_topk(xh, qh, k):
    """Exact L2sq top-k of integer rows, (distance, row) order, in numpy: |x|^2 + |q|^2 -
    2 x.q with every term an integer below 2^24 (exact in f32 whatever BLAS sums first);
    ties broken by row through a composite int64 key (distance * 2^24 + row)."""
    sqx = np.einsum("ij,ij->i", xh, xh)
    sqq = np.einsum("ij,ij->i", qh, qh)
    best = np.full((qh.shape[0], 0), np.iinfo(np.int64).max, np.int64)
    step = 1 << 18
    for lo in range(0, xh.shape[0], step):
        xc = xh[lo:lo + step]
        d = sqq[:, None] + sqx[None, lo:lo + step] - 2.0 * (qh @ xc.T)
        comp = d.astype(np.int64) * (1 << 24) + (np.arange(xc.shape[0], dtype=np.int64) + lo)[None, :]
        part = np.partition(comp, k - 1, axis=1)[:, :k]
        best = np.sort(np.concatenate([best, part], 1), axis=1)[:, :k]
    return best & ((1 << 24) - 1), (best >> 24).astype(np.float32)


@pytest.mark.timeout(900)
def test_c4_full_shard_recall_and_exact_vs_numpy():
    import torch
    n, nq, nq_np = 12_500_000, 10_000, 1000
    assert n < (1 << 24)  # composite key of _numpy_topk
    x = vsg.datagen_device("sift", n, DIM, BS, MS)
    q = vsg.datagen_device("sift", nq, DIM, QS, MS)
    idx = vsg.Index(DIM, "l2sq", "f16", M, EFC, 64, seed=0x5EED)
    idx.reserve(n)
    idx.add_device(np.arange(n, dtype=np.uint64), x)
    assert idx.size() == n
    gk, gd = idx.search_device(q, K, exact=True)
    hk, _ = idx.search_device(q, K, 192)
    torch.cuda.synchronize()
    gt = gk.cpu().numpy().view(np.uint64)
    r = recall(hk.cpu().numpy().view(np.uint64), gt)
    print(f"C4 shard 12.5M x 128 f16: recall@10 at ef 192 = {r:.4f} (10,000 queries)")
    assert r >= 0.95
    xh = x.cpu().numpy()
    qh = q[:nq_np].cpu().numpy()
    del x
    assert np.all(xh == np.rint(xh)) and xh.max() <= 255  # the datagen kernel's rows are integer
    nk, nd = _numpy_topk(xh, qh, K)
    np.testing.assert_array_equal(gt[:nq_np], nk.astype(np.uint64))
    np.testing.assert_array_equal(gd.cpu().numpy()[:nq_np], nd)
