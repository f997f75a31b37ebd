"""The shipped libphx.so's device code, checked from the binary itself (CPU only: llvm-objdump).

* No packed-FP32 VALU instruction (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32) in any gfx950 code
  object.  A bf16 residual add whose v_pk_add_f32 read the high half of a v_pk_mul_f32 result one wait
  state later produced stale values for 16-lane groups while another kernel shared the CU (DESIGN.md
  section 12).  The Makefile default NOPK=1 builds without them; this test is the guard against a build
  that re-admits them (NOPK=0, a TU built outside the Makefile, a compiler that ignores the feature).
* The matrix cores are used: fp32 and bf16 MFMA instructions are present.
* The work-skipping timing knobs are compiled out (make DEBUG_KNOBS=1 builds them in): the names they
  are read under do not occur in the library.
"""
import os
import re
import shutil
import struct
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mladversarialobjectdetection_amd", "libphx.so")
LLVM = "/opt/rocm/lib/llvm/bin"
OBJCOPY = os.path.join(LLVM, "llvm-objcopy")
OBJDUMP = os.path.join(LLVM, "llvm-objdump")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

pytestmark = pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)),
                                reason="needs the built libphx.so and llvm-objdump")


def _code_objects(tmp):
    """Every gfx950 code object of the .hip_fatbin section (clang offload bundles, one per TU)."""
    fb = os.path.join(tmp, "fatbin.bin")
    subprocess.run([OBJCOPY, "--dump-section", f".hip_fatbin={fb}", LIB, os.path.join(tmp, "lib.copy")],
                   check=True, capture_output=True)
    data = open(fb, "rb").read()
    objs, pos = [], 0
    while True:
        b = data.find(MAGIC, pos)
        if b < 0:
            break
        n = struct.unpack_from("<Q", data, b + len(MAGIC))[0]
        p = b + len(MAGIC) + 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                path = os.path.join(tmp, f"co{len(objs)}.o")
                with open(path, "wb") as f:
                    f.write(data[b + off:b + off + size])
                objs.append(path)
        pos = b + 1
    return objs


@pytest.fixture(scope="module")
def disasm():
    tmp = tempfile.mkdtemp()
    try:
        objs = _code_objects(tmp)
        text = []
        for o in objs:
            r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", o], check=True, capture_output=True, text=True)
            text.append(r.stdout)
        yield objs, "\n".join(text)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def test_code_objects_present(disasm):
    objs, _ = disasm
    assert len(objs) >= 10, f"only {len(objs)} gfx950 code objects in {LIB}"


def test_no_packed_fp32_valu(disasm):
    _, text = disasm
    hits = re.findall(r"\bv_pk_(?:add|mul|fma)_f32\b", text)
    assert not hits, f"{len(hits)} packed-FP32 instructions in the shipped device code (build with NOPK=1)"


def test_matrix_cores_used(disasm):
    _, text = disasm
    f32 = len(re.findall(r"\bv_mfma_f32_(?:32x32x2|16x16x4)_f32\b", text))
    bf16 = len(re.findall(r"\bv_mfma_f32_(?:32x32x16|16x16x32)_bf16\b", text))
    assert f32 > 1000 and bf16 > 100, (f32, bf16)


def test_work_skipping_knobs_compiled_out():
    blob = open(LIB, "rb").read()
    for name in (b"PHX_SKIP_TIMING", b"PHX_SKIP_KINDS", b"PHX_NO_DROP"):
        assert name not in blob, f"{name.decode()} is read by the shipped library (built with DEBUG_KNOBS=1?)"


@pytest.mark.parametrize("knob", ["PHX_SKIP_TIMING", "PHX_SKIP_KINDS", "PHX_NO_DROP"])
def test_bench_refuses_work_skipping_knobs(knob):
    """bench.py prints no headline when a knob that skips work is set (it exits before any device
    work, so this runs on CPU); the knobs exist only in a DEBUG_KNOBS=1 build anyway."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, **{knob: "1"})
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode != 0
    assert knob in r.stderr and "no headline" in r.stderr
    assert not r.stdout.strip()
