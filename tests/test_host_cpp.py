"""CPU: host-side C++ logic of libvsg compiled with g++ (no GPU)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_keymap_differential(tmp_path):
    exe = tmp_path / "test_keymap"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", os.path.join(ROOT, "tests", "cpp", "test_keymap.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")


def test_actor_host_logic(tmp_path):
    """csrc/actor.hpp against a mock backend: FIFO add/replace/remove, batched
    concurrent anns equal to single-query answers, ef grouping, capacity
    growth rule (src/index/usearch.rs:200-212), swallowed add errors."""
    exe = tmp_path / "test_actor"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", os.path.join(ROOT, "tests", "cpp", "test_actor.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")
