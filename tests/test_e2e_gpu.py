"""End-to-end parity on the MI355X against the REAL reference's outputs
(tests/golden/golden_e2e.npz / golden_text.npz, produced by
tests/golden/make_golden.py from /root/reference on oracle/synth.py weights).

Contract (BASELINE.json north_star): anomaly maps within 1e-3 abs + 1e-2 rel
(fp32 tolerance), argmax labels bit-exact. Labels are compared where the
reference's own margin exceeds the kernel's rounding (|A1 - A0| > 1e-3 on
the 100x scale, i.e. cos-sim margins > 1e-5) — closer margins are ties at
fp32 resolution and are reported, not asserted.
"""
import numpy as np
import pytest
import torch

from aaclip.engine import TextEngine, VisualEngine
from oracle import synth

pytestmark = pytest.mark.gpu

# bf16 patch-label flips against the reference goldens where its margin exceeds 1e-3 (the
# measured counts, round 4; the tests hold them to twice that)
BF16_FLIPS_336, BF16_FLIPS_336_LEVEL = 6, (0, 4, 2, 0)
BF16_FLIPS_518, BF16_FLIPS_518_LEVEL = 4, (1, 2, 1, 0)
BF16_FLIPS_QUICK = 1  # of 2303 (QuickGELU towers, golden_quick)


@pytest.fixture(scope="module")
def weights(dev):
    sd = synth.clip_state_dict(111)
    ia, ta = synth.adapter_state_dicts(111)
    t = lambda d: {k: torch.from_numpy(v).to(dev) for k, v in d.items()}  # noqa: E731
    return t(sd), t(ia), t(ta), sd


def _visual(weights, dtype, **kw):
    sd, ia, _, _ = weights
    vp = {k: v for k, v in sd.items() if k.startswith("visual.")}
    return VisualEngine(vp, ia, dtype=dtype, **kw)


def _check_e2e(eng, golden, dev, map_tol):
    e = golden["e2e"]
    x = torch.from_numpy(synth.images(111, 2, 336)).to(dev)
    T = torch.from_numpy(e["T"]).to(dev)
    seg, det = eng.forward(x)
    grid = np.stack([(100.0 * (f @ T)).cpu().numpy() for f in seg], axis=1)
    ref_grid = e["grid_A"]
    # labels: argmax over (normal, abnormal) per patch and level
    margin = np.abs(ref_grid[..., 1] - ref_grid[..., 0])
    sure = margin > 1e-3
    lab, ref_lab = grid.argmax(-1), ref_grid.argmax(-1)
    flips_sure = int((lab != ref_lab)[sure].sum())
    maps, score = eng.predict(x, T, "Industrial")
    maps = maps.cpu().numpy()
    atol, rtol = map_tol
    err = np.abs(maps[0] - e["map_ind0"])
    bound = atol + rtol * np.abs(e["map_ind0"])
    ok = bool((err <= bound).all())
    np.testing.assert_allclose(score.cpu().numpy(), e["score"], atol=1e-3)
    np.testing.assert_allclose(det.cpu().numpy(), e["det"], atol=2e-3, rtol=2e-2)
    per_level = [int((lab != ref_lab)[:, lv][sure[:, lv]].sum()) for lv in range(lab.shape[1])]
    return dict(map_max_abs=float(err.max()), map_ok=ok, flips_sure=flips_sure, n_sure=int(sure.sum()),
                flips_sure_per_level=per_level,
                flips_all=int((lab != ref_lab).sum()), grid_max_abs=float(np.abs(grid - ref_grid).max()))


def test_visual_fp32_parity(dev, golden, weights):
    """fp32 parity mode (fp32 MFMA GEMMs + fp32 attention): the strict contract."""
    r = _check_e2e(_visual(weights, torch.float32), golden, dev, (1e-3, 1e-2))
    print("fp32:", r)
    assert r["map_ok"], r
    assert r["flips_sure"] == 0, r
    assert r["grid_max_abs"] < 1e-2, r


def test_visual_bf16_parity(dev, golden, weights):
    """bf16 perf path (bf16 MFMA, fp32 accumulate/residual/softmax/map)."""
    eng = _visual(weights, torch.bfloat16)
    r = _check_e2e(eng, golden, dev, (1e-3, 1e-2))
    print("bf16:", r)
    assert r["map_ok"], r
    # bf16 operands (8 significant bits) can flip a patch label whose margin is within
    # their rounding: reported, and held to a regression bound of twice the measured count
    # (round 4: 6 of 4597 sure labels, per level [0, 4, 2, 0]; the contract mode, fp16,
    # has 0: tests/test_fp16_gpu.py) -- a kernel change that doubles them fails here
    assert r["flips_sure"] <= 2 * BF16_FLIPS_336, r
    assert all(f <= 2 * m + 2 for f, m in zip(r["flips_sure_per_level"], BF16_FLIPS_336_LEVEL)), r
    e = golden["e2e"]
    x = torch.from_numpy(synth.images(111, 2, 336)).to(dev)
    T = torch.from_numpy(e["T"]).to(dev)
    maps, _ = eng.predict(x, T, "Medical")
    np.testing.assert_allclose(maps.cpu().numpy()[:, ::7, ::7], e["map_med_sub"], atol=1e-3, rtol=1e-2)
    # image-level labels (score > 0.5) must agree exactly
    _, score = eng.predict(x, T, "Industrial")
    assert np.array_equal(score.cpu().numpy() > 0.5, e["score"] > 0.5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_text_anchor_parity(dev, golden, weights, dtype):
    sd, _, ta, _ = weights
    tx = golden["text"]
    tp = {k: v for k, v in sd.items() if not k.startswith("visual.")}
    # fp32 mode: fp32 MFMA end to end; bf16 mode: bf16 operands (2^-8 relative) through 12 blocks
    enc_tol, t_tol = (1e-5, 1e-5) if dtype == torch.float32 else (5e-2, 5e-3)
    for adapted, key in ((True, "adapted"), (False, "clip")):
        eng = TextEngine(tp, ta if adapted else None, dtype=dtype)
        enc = eng.encode(torch.from_numpy(tx["bottle_tok_abnormal"]).to(dev)).cpu().numpy()
        ref = tx[f"bottle_enc_abnormal_{key}"]
        np.testing.assert_allclose(enc, ref, atol=enc_tol * max(1.0, np.abs(ref).max()), rtol=enc_tol * 10)
        for cls in ("bottle", "brain"):
            T = eng.class_anchor(torch.from_numpy(tx[f"{cls}_tok_normal"]).to(dev),
                                 torch.from_numpy(tx[f"{cls}_tok_abnormal"]).to(dev)).cpu().numpy()
            np.testing.assert_allclose(T, tx[f"{cls}_T_{key}"], atol=t_tol, rtol=t_tol * 10)


@pytest.mark.parametrize("dtype,scope", [(torch.float32, None), (torch.bfloat16, None),
                                         (torch.float8_e4m3fn, "mlp"), (torch.float8_e4m3fn, "all")])
def test_c5_shapes_parity(dev, golden, dtype, scope):
    """448 px (1025 tokens), 6 levels, relu projections: map vs the reference's golden.
    float8_e4m3fn = config C5's fp8 MFMA mode (block GEMMs on e4m3 weights/activations):
    held to a documented looser bound, since e4m3 (3 mantissa bits) cannot meet the fp32
    contract; its measured error is printed."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_c5.npz"))
    lv = tuple(int(v) for v in g["levels"])
    sd = synth.clip_state_dict(111, img_size=448)
    ia, _ = synth.adapter_state_dicts(111, relu=True, n_levels=len(lv))
    vp = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    kw = dict(fp8_scope=scope) if scope else {}
    eng = VisualEngine(vp, {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}, levels=lv, dtype=dtype, **kw)
    T = torch.from_numpy(golden["text"]["bottle_T_adapted"]).to(dev)
    x = torch.from_numpy(synth.images(111, 1, 448)).to(dev)
    maps, score = eng.predict(x, T, "Medical")
    ref = g["map_med_sub"]
    got = maps.cpu().numpy()[:, ::8, ::8]
    err = np.abs(got - ref)
    print(dtype, "c5 map max abs err", err.max())
    if dtype == torch.float32:
        assert err.max() < 1e-4
        seg, det = eng.forward(x)
        grid = np.stack([(100.0 * (f @ T)).cpu().numpy() for f in seg], axis=1)
        np.testing.assert_allclose(grid, g["grid_A"], atol=5e-3)
    elif dtype == torch.bfloat16:
        assert (err <= 3e-3 + 1.5e-2 * np.abs(ref)).all()
    else:
        rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        within = np.mean(err <= 1e-3 + 1e-2 * np.abs(ref))
        print(f"fp8 ({scope}) c5: map rel-L2 {rel:.3e}, frac within fp32 contract {within:.4f}, "
              f"score err {np.abs(score.cpu().numpy() - g['score']).max():.2e}")
        assert rel < (0.05 if scope == "all" else 0.03)  # measured 2.5-3.8 % / 1.8 %
        np.testing.assert_allclose(score.cpu().numpy(), g["score"], atol=2e-2)
        return
    np.testing.assert_allclose(score.cpu().numpy(), g["score"], atol=1e-3)


def test_graphed_predict_matches_eager(dev, weights):
    """hipGraph replay (incl. the two-stream fork/join) gives bit-identical results."""
    eng = _visual(weights, torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(3)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    for B, streams in ((1, 1), (4, 2)):
        x = torch.randn(B, 3, 336, 336, device=dev, generator=g)
        m0, s0 = [t.clone() for t in eng.predict(x, T, "Industrial", streams=streams)]
        run = eng.graphed_predict(B, 336, "Industrial", streams=streams)
        for _ in range(2):
            m1, s1 = run(x, T)
            torch.cuda.synchronize()
            assert torch.equal(m1, m0) and torch.equal(s1, s0)
        x2 = torch.randn(B, 3, 336, 336, device=dev, generator=g)
        m2, _ = run(x2, T)
        m2 = m2.clone()
        m3, _ = eng.predict(x2, T, "Industrial", streams=streams)
        assert torch.equal(m2, m3)


@pytest.mark.parametrize("dtype,scope", [(torch.bfloat16, "mlp"), (torch.float8_e4m3fn, "mlp"),
                                         (torch.float8_e4m3fn, "all")])
def test_batch_composition_invariance(dev, weights, dtype, scope):
    """Images are independent units: every per-row kernel (GEMM rows, LayerNorm rows,
    per-(image, head) attention, per-image maps/scores) computes the same bits for an
    image whatever the batch size, its position in the batch and the stream chunking
    (size-independent property backing the B=32 bench line and the image sharding);
    uneven explicit chunk splits and a graph captured over them included."""
    eng = _visual(weights, dtype, fp8_scope=scope)
    g = torch.Generator(device=dev).manual_seed(9)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    x = torch.randn(7, 3, 336, 336, device=dev, generator=g)
    ref_m, ref_s = [], []
    for i in range(7):
        m, s = eng.predict(x[i:i + 1], T, "Industrial", streams=1)
        ref_m.append(m.clone())
        ref_s.append(s.clone())
    ref_m, ref_s = torch.cat(ref_m), torch.cat(ref_s)
    for B, streams in ((7, 1), (7, 2), (7, 3), (5, 2), (3, 4), (7, (2, 5)), (7, (4, 1, 2))):
        idx = torch.arange(7 - B, 7, device=dev) if B == 5 else torch.arange(B, device=dev)
        m, s = eng.predict(x[idx], T, "Industrial", streams=streams)
        assert torch.equal(m, ref_m[idx]), (B, streams)
        assert torch.equal(s, ref_s[idx]), (B, streams)
    run = eng.graphed_predict(7, 336, "Industrial", streams=(3, 4))
    eng.predict(x[:2], T, "Industrial", streams=1)  # other batch sizes in between must not disturb the graph
    m, s = run(x, T)
    assert torch.equal(m, ref_m) and torch.equal(s, ref_s)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_text_encode_sequence_invariance(dev, golden, weights, dtype):
    """Prompts are independent sequences: encoding 10 prompts at once gives each the
    same bits as encoding it alone or inside an odd-sized subset (causal attention
    per sequence, row-independent GEMM / LayerNorm rows)."""
    sd, _, ta, _ = weights
    tp = {k: v for k, v in sd.items() if not k.startswith("visual.")}
    eng = TextEngine(tp, ta, dtype=dtype)
    tok = torch.from_numpy(golden["text"]["bottle_tok_abnormal"]).to(dev)
    full = eng.encode(tok).clone()
    for i in (0, 4, tok.shape[0] - 1):
        assert torch.equal(eng.encode(tok[i:i + 1]), full[i:i + 1]), i
    assert torch.equal(eng.encode(tok[3:6]), full[3:6])


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_518_default_size_parity(dev, dtype):
    """518 px (the reference's default, test.py:111): 37x37 grid, 1370-token attention
    (key tail of 26 in a masked tile), 518-wide maps, vs the reference's golden.
    fp32 and fp16 meet the north_star contract on every sampled pixel; bf16 is held to
    the looser bound its 8-bit operands allow."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_518.npz"))
    sd = synth.clip_state_dict(111, img_size=518)
    ia, _ = synth.adapter_state_dicts(111)
    vp = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    eng = VisualEngine(vp, {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}, dtype=dtype)
    x = torch.from_numpy(synth.images(111, 1, 518)).to(dev)
    T = torch.from_numpy(g["T"]).to(dev)
    for dom in ("Industrial", "Medical"):
        maps, score = eng.predict(x, T, dom)
        m = maps.cpu().numpy()
        for got, ref in ((m[:, ::7, ::7], g[f"map_{dom}_sub"]), (m[:, [0, 1, 258, 517], :], g[f"map_{dom}_rows"])):
            err = np.abs(got - ref)
            print(dtype, dom, "518 map max abs err", err.max())
            if dtype == torch.bfloat16:
                assert (err <= 3e-3 + 1.5e-2 * np.abs(ref)).all()
            else:
                assert (err <= 1e-3 + 1e-2 * np.abs(ref)).all()
        np.testing.assert_allclose(score.cpu().numpy(), g["score"], atol=1e-4 if dtype != torch.bfloat16 else 1e-3)
    # patch labels (argmax over the 2 anchors per level and patch) where the reference's
    # margin exceeds 1e-3 on the x100 scale: exact in fp32 and fp16 (the contract mode),
    # reported and bounded in bf16
    seg, det = eng.forward(x)
    grid = np.stack([(100.0 * (f @ T)).cpu().numpy() for f in seg], axis=1)
    ref = g["grid_A"]
    sure = np.abs(ref[..., 1] - ref[..., 0]) > 1e-3
    fl = grid.argmax(-1) != ref.argmax(-1)
    flips = int(fl[sure].sum())
    per_level = [int(fl[:, lv][sure[:, lv]].sum()) for lv in range(fl.shape[1])]
    print(dtype, f"518 patch-label flips (sure) {flips}/{int(sure.sum())} per level {per_level}")
    if dtype == torch.bfloat16:  # measured 4 of 5469 (per level [1, 2, 1, 0]): twice that bounds it
        assert flips <= 2 * BF16_FLIPS_518, (flips, per_level)
        assert all(f <= 2 * m + 2 for f, m in zip(per_level, BF16_FLIPS_518_LEVEL)), per_level
    else:
        assert flips == 0
    if dtype == torch.float32:
        np.testing.assert_allclose(grid, ref, atol=5e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_text_encode_truncation_is_exact(dev, golden, weights, dtype):
    """TextEngine.encode drops the token columns after the longest prompt's EOT (the tower
    is causal): bit-identical to running all 77 columns, adapted and unadapted, for one
    class's prompts and for a mixed-length batch."""
    sd, _, ta, _ = weights
    tp = {k: v for k, v in sd.items() if not k.startswith("visual.")}
    t = golden["text"]
    tok = torch.cat([torch.from_numpy(t["bottle_tok_abnormal"]), torch.from_numpy(t["brain_tok_normal"])]).to(dev)
    for ad in (ta, None):
        eng = TextEngine(tp, ad, dtype=dtype)
        full = eng.encode(tok, truncate=False).clone()
        assert int(tok.argmax(-1).max()) + 1 < tok.shape[1]  # the case actually truncates
        assert torch.equal(eng.encode(tok), full)
        assert torch.equal(eng.encode(tok[:3]), full[:3])


def test_predict_cached_replays_graph_bit_identical(dev, weights):
    """VisualEngine.predict_cached (AdaptedCLIP.predict): eager until a shape follows a
    call of the same shape (a class's full batches), which captures; replayed after --
    every call bit-identical to predict(), with new images and anchors each time.
    Interleaved shapes (a tail batch between classes) never capture; once captured,
    interleaving replays both graphs."""
    eng = _visual(weights, torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(21)

    def call(B, streams, tag):
        x = torch.randn(B, 3, 336, 336, device=dev, generator=g)
        T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
        m1, s1 = (t.clone() for t in eng.predict_cached(x, T, "Industrial", streams=streams))
        m0, s0 = eng.predict(x, T, "Industrial", streams=streams)
        assert torch.equal(m1, m0) and torch.equal(s1, s0), (tag, B)

    shapes = ((4, 2), (2, 1))
    for rep in range(3):  # interleaved: never back to back, so nothing is captured
        for B, streams in shapes:
            call(B, streams, ("interleaved", rep))
    assert len(getattr(eng, "_graph_cache", {})) == 0
    for B, streams in shapes:  # back to back: the second call captures, the third replays
        for rep in range(3):
            call(B, streams, ("repeat", rep))
    assert len(eng._graph_cache) == 2
    for rep in range(2):  # interleaved again: both graphs replay (LRU keeps them)
        for B, streams in shapes:
            call(B, streams, ("replay", rep))
    assert len(eng._graph_cache) == 2


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_quick_gelu_towers_parity(dev, weights, dtype):
    """Towers built with force_quick_gelu=True (reference clip.py:151-153): QuickGELU
    fused into every c_fc epilogue, visual and text, vs the reference's golden_quick.npz.
    fp32 / fp16 hold the map contract (1e-3 + 1e-2 |ref|) with 0 sure-margin label
    flips; bf16 the bf16 bound of the 518 / C5 tests (3e-3 + 1.5e-2 |ref|; measured max
    abs 5.4e-3) with flips bounded as test_visual_bf16_parity."""
    import os
    q = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_quick.npz"))
    eng = _visual(weights, dtype, quick_gelu=True)
    x = torch.from_numpy(synth.images(111, 1, 336)).to(dev)
    T = torch.from_numpy(q["T"]).to(dev)
    seg, det = eng.forward(x)
    grid = np.stack([(100.0 * (f @ T)).cpu().numpy() for f in seg], axis=1)
    sure = np.abs(q["grid_A"][..., 1] - q["grid_A"][..., 0]) > 1e-3
    flips = int((grid.argmax(-1) != q["grid_A"].argmax(-1))[sure].sum())
    maps, score = eng.predict(x, T, "Industrial")
    got = maps.cpu().numpy()[:, ::7, ::7]
    err = np.abs(got - q["map_ind_sub"])
    print(dtype, "quick_gelu map max abs", err.max(), "flips", flips, "of", int(sure.sum()))
    # bf16: the bound the bf16 mode is held to at 518 / C5 (its operands round at 2^-8)
    atol, rtol = (1e-3, 1e-2) if dtype != torch.bfloat16 else (3e-3, 1.5e-2)
    assert (err <= atol + rtol * np.abs(q["map_ind_sub"])).all()
    np.testing.assert_allclose(score.cpu().numpy(), q["score"], atol=1e-3)
    assert flips <= (0 if dtype != torch.bfloat16 else 2 * max(1, BF16_FLIPS_QUICK))
    # the erf-GELU engine on the same weights is visibly off this golden (in bf16 the
    # activation swap moves the map by 1.5e-2 against bf16's own 5e-3: a factor 2.5 there)
    plain = _visual(weights, dtype).predict(x, T, "Industrial")[0].cpu().numpy()[:, ::7, ::7]
    factor = 10 if dtype != torch.bfloat16 else 2.5
    assert np.abs(plain - q["map_ind_sub"]).max() > factor * max(err.max(), 1e-4)
    if dtype == torch.float16:
        return
    sd, _, ta, _ = weights
    tp = {k: v for k, v in sd.items() if not k.startswith("visual.")}
    tol = 1e-5 if dtype == torch.float32 else 5e-2
    for ad, key in ((ta, "adapted"), (None, "clip")):
        enc = TextEngine(tp, ad, dtype=dtype, quick_gelu=True).encode(torch.from_numpy(q["tok_abnormal"]).to(dev))
        ref = q[f"enc_abnormal_{key}"]
        np.testing.assert_allclose(enc.cpu().numpy(), ref, atol=tol * max(1.0, np.abs(ref).max()), rtol=tol * 10)
