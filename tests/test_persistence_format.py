"""Index file format (include/vsg.h "Persistence") checked on CPU: a file
written here from the documented layout is accepted by vsg_index_file_info, and
every kind of damage is rejected before any device is touched."""
import struct

import numpy as np
import pytest

import vsg
from vsg._lib import VsgError

MAGIC = b"VSGIDX\x00\x01"


def fnv(data: bytes, h: int = 0xcbf29ce484222325) -> int:
    for b in data:
        h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def write_file(path, dim=8, metric=2, quant=0, M=4, slots=5, live=4, upper_rows=2, payload_damage=False,
               version=2, entry=0, max_level=1, keys=None, levels=None, adj0=None, upper_off=None, upper=None,
               ring=None):
    """A checksum-valid index file from the documented layout; every section can be
    overridden (crafted graphs for the load-time validation tests).  Version 2 ends with
    the free ring: (slots - live) u32, oldest removal first (default: the removed slots,
    here the first slots - live, ascending)."""
    row_bytes = ((dim * (4 if quant == 0 else 2) + 15) // 16) * 16
    opt = struct.pack("<6IiIQ", dim, metric, quant, M, 32, 16, 0, 0, 7)
    assert len(opt) == 40
    rng = np.random.default_rng(0)
    flags = np.zeros(slots, np.uint8)
    flags[: slots - live] = 1
    sections = [
        rng.standard_normal(slots * row_bytes // 4).astype(np.float32).tobytes(),  # rows
        np.ones(slots, np.float32).tobytes(),  # |x|^2
        (np.arange(slots, dtype=np.uint64) if keys is None else np.asarray(keys, np.uint64)).tobytes(),
        flags.tobytes(),
        (np.zeros(slots, np.int8) if levels is None else np.asarray(levels, np.int8)).tobytes(),
        (np.full(slots * 2 * M, 0xFFFFFFFF, np.uint32) if adj0 is None else np.asarray(adj0, np.uint32)).tobytes(),
        (np.full(slots, 0xFFFFFFFF, np.uint32) if upper_off is None else np.asarray(upper_off, np.uint32)).tobytes(),
        (np.zeros(upper_rows * M, np.uint32) if upper is None else np.asarray(upper, np.uint32)).tobytes(),
    ]
    if version >= 2:
        sections.append((np.arange(slots - live, dtype=np.uint32) if ring is None
                         else np.asarray(ring, np.uint32)).tobytes())
    payload = b"".join(sections)
    head = MAGIC + struct.pack("<II", version, 128) + opt + struct.pack(
        "<4Q4IIiQ", slots, live, upper_rows, row_bytes, M, 2 * M, 32, 16, entry, max_level, fnv(payload))
    head += struct.pack("<Q", fnv(head))
    assert len(head) == 128
    if payload_damage:
        payload = payload[:-1] + bytes([payload[-1] ^ 1])
    with open(path, "wb") as f:
        f.write(head + payload)
    return len(head) + len(payload)


def test_file_info_reads_documented_layout(tmp_path):
    p = tmp_path / "a.vsg"
    n = write_file(p)
    info = vsg.file_info(p)
    assert info["dimensions"] == 8 and info["metric"] == "cos" and info["quantization"] == "f32"
    assert info["connectivity"] == 4 and info["slots"] == 5 and info["live"] == 4
    assert info["upper_rows"] == 2 and info["file_bytes"] == n and info["version"] == 2
    assert info["max_level"] == 1 and info["seed"] == 7
    # payload damage is only detectable by a full read (vsg_index_load), not the header check
    write_file(p, payload_damage=True)
    assert vsg.file_info(p)["slots"] == 5


@pytest.mark.parametrize("damage", ["magic", "header_byte", "truncate", "extra", "version", "empty"])
def test_file_info_rejects_damage(tmp_path, damage):
    p = tmp_path / "b.vsg"
    if damage == "version":
        write_file(p, version=3)
        with pytest.raises(VsgError, match="version"):
            vsg.file_info(p)
        return
    write_file(p)
    raw = bytearray(p.read_bytes())
    if damage == "magic":
        raw[0] ^= 0xFF
    elif damage == "header_byte":
        raw[60] ^= 1  # inside `slots`
    elif damage == "truncate":
        raw = raw[:-3]
    elif damage == "extra":
        raw += b"\0"
    elif damage == "empty":
        raw = b""
    p.write_bytes(bytes(raw))
    with pytest.raises(VsgError):
        vsg.file_info(p)


def test_file_info_missing_file(tmp_path):
    with pytest.raises(VsgError, match="cannot open"):
        vsg.file_info(tmp_path / "nope.vsg")


def test_file_info_reads_version_1(tmp_path):
    """Round-4 files (no free ring) still load: the removed slots become the ring,
    ascending (vsg_index_load)."""
    p = tmp_path / "v1.vsg"
    n = write_file(p, version=1)
    info = vsg.file_info(p)
    assert info["version"] == 1 and info["file_bytes"] == n
    # a version-1 layout labelled version 2 lacks the ring section: size mismatch
    raw = bytearray(p.read_bytes())
    write_file(p, version=2)
    assert len(p.read_bytes()) == len(raw) + 4  # slots - live = 1 ring entry
