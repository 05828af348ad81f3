"""The Rust side of the drop-in (rust/, source only: no cargo/rustc in the image).

CPU: every function rust/src/index/vsg_sys.rs declares is exported by libvsg.so and every
symbol include/vsg.h declares is bound there; the #[repr(C)] structs have the header's field
order (compared with the ctypes mirrors the tests use).
GPU: tests/cpp/test_rust_call_sequence.cpp -- the symbol sequence rust/src/index/gpu.rs
drives (create -> reserve(1M) -> add -> remove+add replace -> search -> count, and the
reference's own unit KAT through the actor, usearch.rs:322-425) -- runs against libvsg.so.
"""
import os
import re
import subprocess

import pytest

import vsg
from vsg import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYS = os.path.join(ROOT, "rust", "src", "index", "vsg_sys.rs")
CPP = os.path.join(ROOT, "tests", "cpp", "test_rust_call_sequence.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_rust_call_sequence")
LIBDIR = os.path.join(ROOT, "vector-store-text_amd", "lib")


def _rust_fns():
    return re.findall(r"pub fn (vsg_\w+)\(", open(SYS).read())


def _rust_struct_fields(name):
    src = open(SYS).read()
    body = re.search(r"pub struct %s \{(.*?)\n\}" % name, src, re.S).group(1)
    return re.findall(r"pub (\w+):", body)


def test_rust_ffi_declares_every_header_symbol_and_all_are_exported():
    fns = _rust_fns()
    assert len(fns) == len(set(fns))
    missing_in_rust = sorted(set(vsg.declared_symbols()) - set(fns))
    assert not missing_in_rust, missing_in_rust
    L = vsg.lib()
    assert not [f for f in fns if not hasattr(L, f)]


@pytest.mark.parametrize("rust,ctype", [("vsg_index_options_t", _lib.Options), ("vsg_stats_t", _lib.Stats),
                                        ("vsg_actor_options_t", _lib.ActorOptions),
                                        ("vsg_actor_counters_t", _lib.ActorCounters),
                                        ("vsg_file_info_t", _lib.FileInfo),
                                        ("vsg_sharded_options_t", _lib.ShardedOptions)])
def test_rust_struct_layouts_match_header(rust, ctype):
    assert _rust_struct_fields(rust) == [f for f, _ in ctype._fields_]


def build_call_sequence() -> str:
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    subprocess.run(["g++", "-O1", "-std=c++17", CPP, "-I", os.path.join(ROOT, "include"), "-L", LIBDIR, "-lvsg",
                    "-Wl,-rpath," + LIBDIR, "-Wl,-rpath-link,/opt/rocm/lib", "-pthread", "-o", EXE], check=True)
    return EXE


def test_call_sequence_driver_compiles(tmp_path):
    assert os.path.exists(build_call_sequence())


@pytest.mark.gpu
@pytest.mark.timeout(120)
def test_rust_call_sequence_on_gpu():
    exe = EXE if os.path.exists(EXE) else build_call_sequence()
    out = subprocess.run([exe], capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("ok")


ROUTES = os.path.join(ROOT, "rust", "src", "httproutes_vector.rs")


def test_rust_vector_routes_match_client_and_python_twin():
    """rust/src/httproutes_vector.rs (source only) serves the client shape of
    /root/reference/tests/integration/httpclient.rs:35-80 with the same paths, request /
    response fields and status mapping as vsg/httproutes.py (which the HTTP tests run)."""
    from vsg import httproutes as H
    src = open(ROUTES).read()
    pairs = re.findall(r'\.route\("([^"]+)",\s*(get|post)\(', src)
    assert pairs == [("/api/v1/indexes", "get"), ("/api/v1/indexes/{keyspace}/{index}/ann", "post"),
                     ("/api/v1/indexes/{keyspace}/{index}/count", "get")]
    assert H.API == "/api/v1"
    req = re.search(r"pub struct PostIndexAnnRequest \{(.*?)\n\}", src, re.S).group(1)
    assert re.findall(r"pub (\w+):", req) == ["embedding", "limit"]
    assert "#[serde(default)]\n    pub limit: Limit" in req      # missing limit -> 1 (Limit::default)
    resp = re.search(r"pub struct PostIndexAnnResponse \{(.*?)\n\}", src, re.S).group(1)
    assert re.findall(r"pub (\w+):", resp) == ["primary_keys", "distances"]
    assert set(H.ann_response(["pk"], [1], [0.5])) == {"primary_keys", "distances"}
    # statuses: unknown index 404 with an empty body, index errors 500 with the error text
    assert src.count('(StatusCode::NOT_FOUND, "")') == 3
    assert 'format!("index.ann request error: {err}")' in src
    assert 'format!("index.count request error: {err}")' in src
    assert "engine.get_index(" in src and "actor.ann(request.embedding, request.limit)" in src
    assert "actor.count()" in src and "engine.get_index_ids()" in src
