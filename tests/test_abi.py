"""The C-ABI library loads on the CPU host and exports every symbol that
include/aaclip.h declares; host-side argument validation rejects bad calls
before any launch (no kernel runs here)."""
import ctypes
import os
import re

import pytest

from aaclip import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "aaclip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(aaclip_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_table():
    assert declared() == sorted(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    for name in declared():
        assert hasattr(lib, name), name
    assert lib.aaclip_abi_version() == _lib.ABI_VERSION
    assert lib.aaclip_arch() == b"gfx950"


def _fake_lib(tmp_path, name, version, symbols=()):
    """A stand-in shared library exporting aaclip_abi_version() (returning `version`) and
    the given no-op symbols: what a stale build of older sources looks like to the loader."""
    import subprocess
    src = tmp_path / f"{name}.c"
    body = f"int aaclip_abi_version(void) {{ return {version}; }}\n" if version is not None else ""
    body += "".join(f"int {s}(void) {{ return 0; }}\n" for s in symbols)
    src.write_text(body or "int unrelated_symbol(void) { return 0; }\n")
    out = tmp_path / f"{name}.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(out), str(src)], check=True)
    return str(out)


def test_stale_library_is_refused_with_one_clear_error(tmp_path):
    """_lib.load checks aaclip_abi_version BEFORE binding anything else (round 5: new Python
    against a stale .so surfaced as AttributeErrors in 20+ tests): a wrong version, a
    right version with missing entry points, and a foreign library each raise ONE
    RuntimeError that names the problem; the real library loads."""
    others = [s for s in _lib.SIGNATURES if s != "aaclip_abi_version"]
    with pytest.raises(RuntimeError, match=r"ABI version 5, this package needs"):
        _lib.load(_fake_lib(tmp_path, "old", 5, others))
    with pytest.raises(RuntimeError, match=r"lacks aaclip_trace_buffer.*stale"):
        _lib.load(_fake_lib(tmp_path, "partial", _lib.ABI_VERSION, [s for s in others if s != "aaclip_trace_buffer"]))
    with pytest.raises(RuntimeError, match=r"exports no aaclip_abi_version"):
        _lib.load(_fake_lib(tmp_path, "foreign", None))
    with pytest.raises(RuntimeError, match=r"missing"):
        _lib.load(str(tmp_path / "absent.so"))
    assert _lib.load(_lib.LIB_PATH).aaclip_abi_version() == _lib.ABI_VERSION


def test_argument_validation_rejects_without_launch():
    lib = _lib.lib()
    # null operands / bad dtype / unsupported shapes return AACLIP_ERR_ARG (=1)
    assert lib.aaclip_gemm(5, 0, 8, 128, 64, None, 64, None, 64, None, 128, 0, None, None, 0, None, 0, 0, 0, 0, None) == 1
    assert lib.aaclip_attention(1, None, None, 1, 8, 1, 64, 0, None, 0, None) == 1
    assert lib.aaclip_attention(1, ctypes.c_void_p(16), ctypes.c_void_p(16), 1, 8, 1, 128, 0, None, 0, None) == 1
    assert lib.aaclip_attention(2, ctypes.c_void_p(16), ctypes.c_void_p(16), 1, 8, 2, 64, 0, None, 0, None) == 1
    assert lib.aaclip_layernorm(0, None, 512, None, None, None, 512, 4, 512, None, 0, None) == 1
    # fp8 MX outputs need their scale buffer; MX GEMM needs its operand scales
    f16 = ctypes.c_void_p(16)
    assert lib.aaclip_layernorm(2, f16, 1024, f16, f16, f16, 1024, 4, 1024, None, 0, None) == 1
    assert lib.aaclip_gemm_fp8mx(0, 8, 256, 128, f16, 128, None, 8, f16, 128, f16, f16, 256, 0, None, None, 0,
                                 None, 0, None, 0, None) == 1
    assert lib.aaclip_quant_fp8_mx(1, f16, 100, f16, 128, f16, 4, 4, 100, None) == 1  # cols % 128
    assert lib.aaclip_blur_upsample(None, None, 1, 3, 24, 336, 7, 1.0, 0, None) == 1
    lv = (ctypes.c_void_p * 1)(16)
    assert lib.aaclip_patch_scores(1, lv, 1, 768, ctypes.c_void_p(16), 4, 512, 1, 0, 0, ctypes.c_void_p(16), None) == 1
    with pytest.raises(RuntimeError):
        _lib.check(1, "aaclip_gemm")
    # the product library has no trace scopes: arming a trace buffer is refused (make trace builds them)
    if not os.environ.get("AACLIP_LIB"):
        assert lib.aaclip_trace_buffer(f16, f16, 16) == 1
        assert lib.aaclip_trace_buffer(None, None, 0) == 1


def test_product_path_does_not_import_the_oracle():
    pkg = os.path.join(ROOT, "aa-clip_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, flags=re.M), f


def test_gemm_plan_per_shape_choice():
    """The default bf16 dispatch's per-shape kernel choice (host logic, no launch):
    fewer tile rounds over 256 CUs, 256-row 8-phase tiles weighted 10/11 -- the
    choices measured fastest per shape."""
    lib = _lib.lib()
    ph8, t320 = "gemm_bf16_8ph_kernel<256,256>", "gemm_bf16_kernel<320,256,2,4>"

    def plan(M, N, K=1024):
        return lib.aaclip_gemm_plan(_lib.BF16, M, N, K).decode()
    # two-stream C2 pipeline: 16 images per stream
    assert [plan(9232, n) for n in (3072, 1024, 4096)] == [ph8, ph8, t320]
    assert plan(9232, 1024, 4096) == ph8  # c_proj
    # whole-batch launches (bench roofline shapes)
    assert [plan(18464, n) for n in (3072, 1024, 4096)] == [ph8, t320, ph8]
    # a few images: 128x128 tiles when the big-tile choice fills under half the CUs
    small, tiny = "gemm_bf16_kernel<128,128,2,2>", "gemm_bf16_kernel<64,64,2,2>"
    # one image: 64x64 tiles where even 128x128 ones number under half the CUs (QKV 120,
    # out-proj / c_proj 40 tiles), 128x128 for c_fc (160)
    assert [plan(577, n) for n in (3072, 1024, 4096)] == [tiny, tiny, small]
    assert plan(577, 1024, 4096) == tiny  # c_proj
    assert [plan(4616, n) for n in (3072, 1024, 4096)] == [ph8, small, t320]
    assert plan(100, 384) == "gemm_bf16_kernel<256,128,4,2>"
    assert lib.aaclip_gemm_plan(_lib.F32, 100, 256, 64) == b"gemm_f32_kernel"


def test_gemm_pin_table_unpins_and_never_fills():
    """aaclip_gemm_pin: unpinning removes the entry, so pinning and unpinning far more
    distinct shapes than the table holds (256) never fails; pins override the
    heuristic and their removal restores it (host logic, no launch)."""
    lib = _lib.lib()
    ph8, t320 = "gemm_bf16_8ph_kernel<256,256>", "gemm_bf16_kernel<320,256,2,4>"
    plan = lambda M, N, K=1024: lib.aaclip_gemm_plan(_lib.BF16, M, N, K).decode()  # noqa: E731
    for rnd in range(3):
        for b in range(1, 301):  # 300 distinct chunk sizes per round
            assert lib.aaclip_gemm_pin(_lib.BF16, b * 577, 4096, 1024, 8) == 0
            assert plan(b * 577, 4096) == t320
            assert lib.aaclip_gemm_pin(_lib.BF16, b * 577, 4096, 1024, 0) == 0
    assert plan(18464, 3072) == ph8  # heuristic again
    # many live pins at once: the table's capacity is reported as an argument error, not UB
    before = plan(1000, 1024)
    rc = [lib.aaclip_gemm_pin(_lib.BF16, 1000 + i, 1024, 1024, 8) for i in range(300)]
    assert rc[:256] == [0] * 256 and set(rc[256:]) == {1}
    for i in range(300):
        assert lib.aaclip_gemm_pin(_lib.BF16, 1000 + i, 1024, 1024, 0) == 0
    assert plan(1000, 1024) == before != t320  # no stale entry left behind
    assert lib.aaclip_gemm_pin(_lib.BF16, 1000, 1024, 1024, 9) == 0
    assert plan(1000, 1024) == "gemm_bf16_kernel<128,128,2,2>"
    assert lib.aaclip_gemm_pin(_lib.BF16, 1000, 1024, 1024, 0) == 0


def test_gemm_concurrent_mode_is_thread_local():
    """aaclip_gemm_concurrent: on the calling thread, shapes whose 256x256 tiles fill a
    round of the 256 CUs take the 8-phase kernel (c_fc at 16 images per chunk), other
    threads keep the heuristic, and the previous state comes back."""
    import threading
    from aaclip import ops
    lib = _lib.lib()
    ph8, t320 = "gemm_bf16_8ph_kernel<256,256>", "gemm_bf16_kernel<320,256,2,4>"
    plan = lambda: lib.aaclip_gemm_plan(_lib.BF16, 9232, 4096, 1024).decode()  # noqa: E731
    assert plan() == t320
    seen = {}
    with ops.concurrent_gemms(True):
        assert plan() == ph8
        assert lib.aaclip_gemm_plan(_lib.BF16, 577, 4096, 1024).decode() != ph8  # under one round: unchanged
        t = threading.Thread(target=lambda: seen.setdefault("other", plan()))
        t.start()
        t.join()
        with ops.concurrent_gemms(False):
            assert plan() == t320
        assert plan() == ph8
    assert plan() == t320 and seen["other"] == t320


def test_tuner_families_are_all_pinnable():
    """Every family ops.tune_gemm tries is one aaclip_gemm_pin accepts (host logic, no
    launch): the removed two-workgroup family 10 is refused and no longer listed."""
    from aaclip import ops
    lib = _lib.lib()
    for fam in ops.GEMM_FAMILIES:
        assert lib.aaclip_gemm_pin(_lib.BF16, 1234, 1024, 1024, fam) == 0, fam
        assert lib.aaclip_gemm_pin(_lib.BF16, 1234, 1024, 1024, 0) == 0
    assert 10 not in ops.GEMM_FAMILIES and lib.aaclip_gemm_pin(_lib.BF16, 1234, 1024, 1024, 10) == 1


def test_gemm_ksplit_argument_validation():
    """aaclip_gemm_ksplit refuses what its grid and workspace cannot take (host logic)."""
    lib = _lib.lib()
    nb, nc = ctypes.c_size_t(0), ctypes.c_int64(0)
    assert lib.aaclip_gemm_ksplit_workspace(9232, 1024, 4096, 3, ctypes.byref(nb), ctypes.byref(nc)) == 0
    assert nb.value == 3 * (9232 + 319) * 1024 * 4 and nc.value == 145 * 16
    assert lib.aaclip_gemm_ksplit_workspace(9232, 1024, 4096, 5, ctypes.byref(nb), ctypes.byref(nc)) == 1
    assert lib.aaclip_gemm_ksplit_workspace(9232, 1024, 128, 3, ctypes.byref(nb), ctypes.byref(nc)) == 1  # 2 K-steps
    f16 = ctypes.c_void_p(16)
    args = [1, 0, 9232, 1024, 4096, f16, 4096, f16, 4096, f16, 1024, 0, None, None, 0, None, 0]
    # workspace too small / split out of range / fp32 operands
    assert lib.aaclip_gemm_ksplit(*args, 3, f16, 1024, f16, 10 ** 6, None) == 1
    assert lib.aaclip_gemm_ksplit(*args, 1, f16, 10 ** 12, f16, 10 ** 6, None) == 1
    assert lib.aaclip_gemm_ksplit(*([0] + args[1:]), 3, f16, 10 ** 12, f16, 10 ** 6, None) == 1
