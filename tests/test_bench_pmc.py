"""CPU: the bench reports a PMC traffic figure only while the committed summary
(profiles/search_pmc.json, build_pmc.json) was profiled on this tree's kernels --
the summary records the source hash it ran (tools/pmc_summary.py) and bench.py
compares it with kernel_src_sha() of the tree."""
import importlib.util
import json
import os
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_search_pmc_used_only_for_the_profiled_kernels(monkeypatch):
    b = _bench()
    d = json.load(open(os.path.join(ROOT, "profiles", "search_pmc.json")))
    w = d["workload"]
    a = SimpleNamespace(rows=w["n"], dim=w["dim"], queries=w["queries"], metric=w["metric"])
    monkeypatch.setattr(b, "kernel_src_sha", lambda: d["kernel_src_sha"])
    assert b.pmc_traffic(a, w["ef"]) == d["hbm_bytes_per_launch"]
    assert b.pmc_traffic(a, w["ef"] + 1) is None  # another workload
    monkeypatch.setattr(b, "kernel_src_sha", lambda: "0" * 16)  # kernels changed since
    assert b.pmc_traffic(a, w["ef"]) is None


def test_kernel_src_sha_tracks_the_sources(tmp_path, monkeypatch):
    b = _bench()
    h0 = b.kernel_src_sha()
    assert len(h0) == 16 and h0 == b.kernel_src_sha()
    # a copy of the tree with one kernel source changed hashes differently
    src = os.path.join(ROOT, "vector-store-text_amd", "csrc")
    dst = tmp_path / "vector-store-text_amd" / "csrc"
    dst.mkdir(parents=True)
    for f in os.listdir(src):
        if f.endswith((".hip", ".hpp", ".cpp")):
            (dst / f).write_bytes(open(os.path.join(src, f), "rb").read())
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    assert b.kernel_src_sha() == h0
    (dst / "hnsw.hip").write_bytes((dst / "hnsw.hip").read_bytes() + b"\n// changed\n")
    assert b.kernel_src_sha() != h0
