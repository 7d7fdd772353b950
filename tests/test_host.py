"""CPU tests of the host side: the C ABI library loads and exports every
symbol include/vame.h declares, the per-POC host logic (lambda, QP, reference
ring) against tests/golden/hostlogic.json, the product geometry against the
oracle, and the work accounting of SURVEY.md §8."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from vame import _lib
from vame.hostlogic import geometry, lambda_for_poc, poc_qp, ref_list
from vame.metrics import pair_accounting

import oracle_py as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(REPO, "tests", "golden", "hostlogic.json")))


def header_symbols():
    src = open(os.path.join(REPO, "include", "vame.h")).read()
    src = re.sub(r"/\*.*?\*/|//[^\n]*", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vame_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 16
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(_lib.EXPORTS) == syms


def test_version_and_errors():
    L = _lib.lib()
    assert b"gfx950" in L.vame_version()
    for code in (0, -1, -2, -3, -4):
        assert L.vame_strerror(code)
    # no device work: bad arguments fail before touching HIP
    assert L.vame_affine_me(None, None, None, 1.0, 0, 2, 0, None, None, None, None) == -1
    assert L.vame_num_ctus(1920, 1080) == 135
    assert L.vame_num_ctus(3840, 2160) == 510
    assert L.vame_cus_per_ctu(0) == 201 and L.vame_cus_per_ctu(1) == 284


def test_work_items_cover_every_cu_once():
    """The engine's work-item templates (vame_create's build_templates, run on
    the host without a device) partition the CTU's candidate CUs: every FULL
    (201) and HALF (284) output offset is covered by exactly one item's CU
    slot -- the 128x128 CU and each 128x64 / 64x128 CU an item of its own;
    per quadrant, affine_me_quad's items (the 64x64 CU cooperative, the
    16-sub-block CUs in autonomous items of 16 wave tasks) and
    affine_me_quad2's (the CUs of 32 to 128 sub-blocks, two stacked
    sub-blocks per lane, in autonomous items), mixing the alignments in a
    launch of both (8 + 8 quadrant items per CTU); the PROF packing (every
    quadrant CU in affine_me_quad) covers alike.  The CTU-item packing of
    rounds 1-5 is gone (half128 = 0 is rejected)."""
    L = _lib.lib()
    items = (ctypes.c_int32 * 3)()
    for align, n in ((0, 201), (1, 284)):
        hits = (ctypes.c_int32 * n)()
        assert L.vame_template_coverage(1, align, hits, items) == 0
        assert list(hits) == [1] * n, (align, [i for i in range(n) if hits[i] != 1])
        assert L.vame_template_coverage(0, align, hits, items) == -1
    quad, ctu, half = list(items)
    assert (quad, ctu, half) == (16, 1, 4)


def test_engine_reads_at_most_five_knobs():
    """the product library reads at most five environment
    variables, each documented in include/vame.h."""
    src = open(os.path.join(os.path.dirname(__file__), "..", "vvc-affine-gpu_amd", "csrc",
                            "vame_engine.hip")).read()
    knobs = set(re.findall(r'env_int\("(VAME_[A-Z_]+)"', src))
    assert src.count("getenv") <= 5 and 0 < len(knobs) <= 5, knobs
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "vame.h")).read()
    for k in knobs:
        assert k in hdr, k


@pytest.mark.parametrize("row", GOLD["lambda"], ids=lambda r: f"qp{r['qp']}_poc{r['poc']}")
def test_lambda_and_qp(row):
    assert poc_qp(row["qp"], row["poc"]) == row["poc_qp"]
    assert np.float32(lambda_for_poc(row["qp"], row["poc"])) == np.float32(row["lambda"])


def test_lambda_kats():
    # SURVEY.md §8a T14
    assert abs(lambda_for_poc(32, 1) - 78.949063) < 1e-5
    assert abs(lambda_for_poc(32, 2) - 70.335619) < 1e-5
    assert abs(lambda_for_poc(32, 8) - 35.167810) < 1e-5


def test_reference_ring():
    for poc, refs in GOLD["ref_lists"].items():
        assert ref_list(int(poc)) == refs, poc


def test_geometry_matches_oracle():
    for align in (0, 1):
        prod = geometry(align)
        ref = O.group_geometry(align)
        assert len(prod) == len(ref)
        for (w, h, xs, ys, s), (w2, h2, xs2, ys2, s2) in zip(prod, ref):
            assert (w, h, s) == (w2, h2, s2)
            assert (xs == xs2).all() and (ys == ys2).all()


def test_pair_accounting_matches_survey():
    a = pair_accounting(1920, 1080, (2,))
    assert a["rows"] == 65475 and a["rows_inframe"] == 60810
    assert a["bytes"] == 2674603500
    b = pair_accounting(1920, 1080, (2, 3))
    assert b["bytes"] == 4918027800
    c = pair_accounting(3840, 2160, (2,))
    assert c["bytes"] == 10811623320
    assert pair_accounting(3840, 2160, (2, 3))["bytes"] == 19880178480


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
@pytest.mark.parametrize("defs", [["-DVAME_ABLATE=63"], ["-DVAME_DUP=23"], ["-DVAME_PHASE_TIMING=1"], ["-DVAME_COUNT_PRED=1"]],
                         ids=["ablate", "dup", "phase", "count"])
def test_instrumentation_builds_compile(tmp_path, defs):
    """The timing-only / profiling builds (make ablate / variant / phase; the
    only compile-time switches the kernel keeps) still compile for gfx950."""
    import subprocess
    src = os.path.join(os.path.dirname(__file__), "..", "vvc-affine-gpu_amd", "csrc", "vame_engine.hip")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17",
                        "-ffp-contract=off", "--cuda-device-only", "-c", *defs, "-o",
                        str(tmp_path / "ab.o"), src], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]


def test_build_record_matches_the_library():
    """__graft_entry__.build() recompiles libvame.so and records its sha256 in
    lib/build_record.json; bench.py reports whether the library it loaded is
    that build's.  A record that no longer matches the library on disk means a
    later build bypassed build() (skipped when no record was written)."""
    import hashlib
    rec_path = os.path.join(os.path.dirname(_lib.LIB_PATH), "build_record.json")
    if not os.path.exists(rec_path) or os.environ.get("VAME_LIB"):
        pytest.skip("no build record (library not built by __graft_entry__.build())")
    rec = json.load(open(rec_path))
    want = rec["artefacts"]["vvc-affine-gpu_amd/lib/libvame.so"]["sha256"]
    assert hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest() == want
    assert rec["mode"].startswith("rebuilt")


def kernel_scratch(lib_path):
    """{kernel: private_segment_fixed_size} from the gfx950 code objects inside
    a built library (the clang offload bundle of each translation unit's fat
    binary, the AMDGPU metadata note read by llvm-readelf)."""
    import struct
    import subprocess
    import tempfile
    d = open(lib_path, "rb").read()
    out_map = {}
    i = d.find(b"__CLANG_OFFLOAD_BUNDLE__")
    assert i >= 0, "no offload bundle in " + lib_path
    while i >= 0:
        n = struct.unpack_from("<Q", d, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, idl = struct.unpack_from("<QQQ", d, p)
            p += 24
            ident = d[p:p + idl].decode()
            p += idl
            if "gfx950" not in ident:
                continue
            with tempfile.NamedTemporaryFile(suffix=".co") as f:
                f.write(d[i + off:i + off + size])
                f.flush()
                out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name],
                                     capture_output=True, text=True, check=True).stdout
            names = re.findall(r"\.name:\s+(\S+)", out)
            priv = [int(v) for v in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", out)]
            assert len(names) == len(priv) and names
            for k, v in zip(names, priv):
                assert k not in out_map, "kernel in two units: " + k
                out_map[k] = v
        i = d.find(b"__CLANG_OFFLOAD_BUNDLE__", i + 32)
    assert out_map, "no gfx950 code object in " + lib_path
    return out_map


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf"), reason="no llvm-readelf")
def test_product_kernels_have_no_scratch():
    """(near-)zero scratch in the product kernels rests on the
    build's flags (-disable-machine-licm; SimplifyCFG's common-code sinking
    off, for the 2-CP-only unit its hoisting too; uniform regions left
    unstructurized -- the Makefile) and on the kernels' opaque()
    recomputation, so a compiler update or a kernel edit that brings spills
    back fails here: the quadrant kernels (affine_me_quad, affine_me_quad2, the
    bulk of every step) have a zero private segment, the 128-class ones at most
    8 B per lane (one slot in affine_me_ctu2<2>, affine_me_half2w/h<2,3>); the
    PROF variants are not the benchmarked path."""
    sizes = kernel_scratch(_lib.LIB_PATH)
    product = {k: v for k, v in sizes.items() if "affine_me" in k and "prof" not in k}
    assert len(product) == 16, sorted(product)
    for k, v in product.items():
        if "affine_me_quad" in k:
            assert v == 0, (k, v)
        else:
            assert v <= 8, (k, v)
