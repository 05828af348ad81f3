"""CPU: libvsg.so loads, exports every symbol include/vsg.h declares, and its
host-only helpers agree with the oracle.  No compute calls (no GPU here)."""
import ctypes as C

import numpy as np

import oracle as O
import vsg
from vsg import _lib


def test_header_symbols_exported():
    declared = vsg.declared_symbols()
    assert len(declared) >= 20
    L = vsg.lib()
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing


def test_all_c_symbols_have_ctypes_signatures():
    L = vsg.lib()
    for s in vsg.declared_symbols():
        f = getattr(L, s)
        assert f.argtypes is not None, s


def test_level_sampling_matches_oracle_bitexact():
    for seed in (0, 1, 0x5EED):
        for m in (2, 8, 16, 32):
            a = [vsg.sample_level(seed, s, m) for s in range(3000)]
            b = [O.sample_level(seed, s, m) for s in range(3000)]
            assert a == b


def test_version_and_error_strings():
    L = vsg.lib()
    assert b"gfx950" in L.vsg_version()
    assert isinstance(L.vsg_last_error(), bytes)


def test_options_struct_layout_matches_header():
    # vsg_index_options_t: 8 x u32/i32 + u64 = 40 bytes
    assert C.sizeof(_lib.Options) == 40
    # vsg_stats_t: the header's uint64_t fields, in order, are the ctypes mirror's
    import re
    txt = open(_lib.HEADER).read()
    body = txt[:txt.index("} vsg_stats_t;")].rsplit("typedef struct {", 1)[1]
    fields = re.findall(r"uint64_t\s+(\w+);", body)
    assert [f for f, _ in _lib.Stats._fields_] == fields
    assert C.sizeof(_lib.Stats) == len(fields) * 8


def test_invalid_options_rejected_without_device():
    # argument validation happens before any device work
    opt = _lib.Options(0, 0, 0, 0, 0, 0, 0, 0, 0)
    h = C.c_void_p()
    rc = vsg.lib().vsg_index_new(C.byref(opt), C.byref(h))
    assert rc == _lib.VSG_EINVAL and not h.value
    assert b"dimensions" in vsg.lib().vsg_last_error()
    opt = _lib.Options(8, 0, 0, 65, 0, 0, 0, 0, 0)  # connectivity: [2, 64]
    rc = vsg.lib().vsg_index_new(C.byref(opt), C.byref(h))
    assert rc == _lib.VSG_EUNSUPPORTED and b"connectivity" in vsg.lib().vsg_last_error()


def test_no_silent_fallback_when_library_missing(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    try:
        _lib.lib()
        raise AssertionError("expected a loud failure")
    except RuntimeError as e:
        assert "no CPU fallback" in str(e)
    finally:
        monkeypatch.setattr(_lib, "_lib", None)


def test_datagen_numpy_deterministic():
    from vsg import datagen as G
    a = G.clustered(64, 32, 1, 2)
    b = G.clustered(64, 32, 1, 2)
    np.testing.assert_array_equal(a, b)
    # prefix / offset consistency
    c = G.clustered(16, 32, 1, 2, start=48)
    np.testing.assert_array_equal(a[48:], c)
    u = G.uint8_valued(100, 16, 5)
    assert u.min() >= 0 and u.max() <= 255 and (u == np.round(u)).all()
