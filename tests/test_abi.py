"""The C-ABI library loads and exports every symbol include/mpx.h declares.

CPU-only: no compute call is made (argument validation that returns before
touching the GPU is allowed).
"""
import ctypes
import ctypes as C
import os
import shutil
import subprocess
import sys

import pytest

import mpx

HERE = os.path.dirname(os.path.abspath(__file__))

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_built_in_tree():
    assert os.path.exists(mpx.LIB_PATH)
    assert mpx.LIB_PATH.startswith(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_every_header_symbol_is_exported():
    syms = mpx.header_symbols()
    assert len(syms) >= 20
    L = ctypes.CDLL(mpx.LIB_PATH)
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    dyn = subprocess.run(["nm", "-D", "--defined-only", mpx.LIB_PATH], capture_output=True, text=True).stdout
    for s in syms:
        assert f" T {s}\n" in dyn or f" T {s}" in dyn, s


def test_counter_library_exports_its_header():
    """libmpxprof.so (bench.py's in-process counters) exports every function
    include/mpxprof.h declares; loading it starts nothing (no HIP here)."""
    from mpx import counters
    hdr = os.path.join(os.path.dirname(mpx.HEADER_PATH), "mpxprof.h")
    import re
    txt = re.sub(r"/\*.*?\*/", "", open(hdr).read(), flags=re.S)
    names = sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_]+\s*\*?\s*(mpxprof_[a-z_]+)\s*\(", txt, flags=re.M)))
    assert names == ["mpxprof_begin", "mpxprof_end", "mpxprof_error", "mpxprof_ready", "mpxprof_register"]
    dyn = subprocess.run(["nm", "-D", "--defined-only", counters.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert f" T {n}" in dyn, n


def test_version_and_strerror():
    L = mpx.lib()
    # 2: recv_done / recv_digest; 3: 64 ranks per context; 4: receive-posted mailbox word;
    # 5: pull mode (MPX_XFER_PULL, tx in the rank descriptor); 6: mpx_last_phases,
    # mpx_device_bus_id, MPX_XFER_NOSTAGE, kernel-cleared scratch words
    assert L.mpx_version() == 7
    texts = {L.mpx_strerror(i).decode() for i in range(9)}
    assert len(texts) == 9
    assert L.mpx_strerror(12345) == b"unknown mpx status"


def test_argument_validation_without_gpu():
    L = mpx.lib()
    h = ctypes.c_void_p()
    assert L.mpx_init(0, 0, ctypes.byref(h)) == mpx.ERR_INVALID
    assert L.mpx_init(mpx.MAX_RANKS + 1, 0, ctypes.byref(h)) == mpx.ERR_INVALID
    assert L.mpx_init(2, 7, ctypes.byref(h)) == mpx.ERR_INVALID
    # SURVEY §8b's HOST engine id is reserved and refused (no CPU transfer path)
    assert L.mpx_init(2, mpx.ENGINE_HOST, ctypes.byref(h)) == mpx.ERR_UNSUPPORTED
    assert b"HOST" in L.mpx_last_error()
    assert L.mpx_finalize(None) == mpx.ERR_INVALID
    assert L.mpx_xfer(None, 0, 1, 0, 1, 1, None, None, 8, None) == mpx.ERR_INVALID
    assert L.mpx_rccl_get_unique_id(None) == mpx.ERR_INVALID
    assert L.mpx_link_info(0, 1, None, None) == mpx.ERR_INVALID
    assert b"NULL" in L.mpx_last_error() or L.mpx_last_error()


def test_header_constants_match_binding():
    txt = open(mpx.HEADER_PATH).read()
    assert "#define MPX_MAX_RANKS 64" in txt and mpx.MAX_RANKS == 64
    assert "#define MPX_RANK_DESC_BYTES 512" in txt
    assert "0x6d70695f70657266ULL" in txt and mpx.PATTERN_SEED == 0x6D70695F70657266
    assert "#define MPX_LINK_XGMI 4" in txt and mpx.LINK_TYPES[4] == "xgmi"
    assert f"#define MPX_ABI_VERSION {mpx.ABI_VERSION}" in txt
    assert f"#define MPX_XFER_STREAM {mpx.XFER_STREAM}" in txt
    assert f"#define MPX_XFER_PULL {mpx.XFER_PULL}" in txt and mpx.PROTOCOLS[7] == "pull"


def test_struct_layouts_match_the_header(tmp_path):
    """Every C struct the binding mirrors (mpx_timing, mpx_xfer_opts,
    mpx_phases) has the binding's size and field offsets: a C program built
    against include/mpx.h prints them (no GPU, no libmpx call)."""
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    mirrors = {"mpx_timing": mpx.Timing, "mpx_xfer_opts": mpx.XferOpts, "mpx_phases": mpx.Phases}
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "mpx.h"', "int main(void) {"]
    for cname, py in mirrors.items():
        src.append(f'    printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            src.append(f'    printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    src += ["    return 0;", "}"]
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src) + "\n")
    exe = tmp_path / "layout"
    inc = os.path.join(ROOT, "include")
    subprocess.run([cc, "-std=c11", "-I", inc, str(c), "-o", str(exe)], check=True, capture_output=True)
    got = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        name, field, val = line.split()
        got[(name, field)] = int(val)
    for cname, py in mirrors.items():
        assert got[(cname, "size")] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_completion_line_layout_and_seal(tmp_path):
    """The kernel engine's call end (mpx_internal.h Fin): one 64-byte,
    64-byte-aligned line inside the host-mapped Status (the kernel writes it
    with a single eight-lane store), and a completion word carrying the
    call token's low 32 bits and a seal that changes with any other field.
    Host-only compile of the internal header (no GPU)."""
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no C++ compiler")
    src = tmp_path / "fin.cpp"
    src.write_text("""#include "mpx_internal.h"
#include <cstddef>
#include <cstdio>
using namespace mpx;
int main() {
    const u64 t = 0x1234567890ull;
    const u64 w = fin_word(t, 1, 2, 3, 4, 5, 6, 7);
    int differ = 1;
    for (int k = 0; k < 7; ++k) {
        u64 v[7] = {1, 2, 3, 4, 5, 6, 7};
        v[k] ^= 1;
        differ &= fin_word(t, v[0], v[1], v[2], v[3], v[4], v[5], v[6]) != w;
    }
    printf("%zu %zu %zu %zu %d %d\\n", sizeof(Fin), alignof(Fin), offsetof(Status, fin) % 64,
           offsetof(Fin, word), (int)((w & 0xffffffffull) == (t & 0xffffffffull)), differ);
    return 0;
}
""")
    exe = tmp_path / "fin"
    subprocess.run([cxx, "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I", os.path.join(ROOT, "mpi-perf_amd", "csrc"), str(src), "-o", str(exe)],
                   check=True, capture_output=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert out == ["64", "64", "0", "56", "1", "1"], out


@pytest.mark.parametrize("torch_first", [False, True])
def test_rccl_is_the_images_whatever_was_loaded_first(torch_first):
    """libmpx binds RCCL at run time from /opt/rocm/lib/librccl.so.1
    (RTLD_LOCAL | RTLD_DEEPBIND), so a process that imported torch first
    (its bundled librccl.so.1 2.26.6 loaded) still runs the image's RCCL,
    as mpx_perf does.  No GPU call: ncclGetVersion."""
    code = ("import sys, json; sys.path.insert(0, %r)\n" % os.path.join(os.path.dirname(HERE), "mpi-perf_amd")
            + ("import torch\n" if torch_first else "")
            + "import mpx; print(json.dumps(mpx.rccl_version()))")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-600:]
    import json
    v = json.loads(r.stdout.strip().splitlines()[-1])
    assert v["library"] == "/opt/rocm/lib/librccl.so.1" and v["release"].startswith("2.27"), v


def test_rccl_unloadable_is_an_error_not_a_fallback(tmp_path):
    """MPX_RCCL_LIB naming a file that cannot be loaded: the RCCL entry points
    fail with MPX_ERR_RCCL and the loader's message."""
    code = ("import sys; sys.path.insert(0, %r)\n" % os.path.join(os.path.dirname(HERE), "mpi-perf_amd")
            + "import mpx\ntry:\n    mpx.rccl_version()\nexcept mpx.MpxError as e:\n"
            + "    print(e.status == mpx.ERR_RCCL, 'cannot load' in str(e))\n")
    env = dict(os.environ, MPX_RCCL_LIB=str(tmp_path / "nope.so"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.stdout.split() == ["True", "True"], (r.stdout, r.stderr[-400:])
