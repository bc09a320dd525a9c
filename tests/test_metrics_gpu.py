"""Device metrics_eval (aaclip_metrics_eval) against the
reference's golden dict and against sklearn's roc_auc_score /
average_precision_score on the same inputs (unrounded, |diff| <= 1e-9): ties,
negative scores, the max == 1 no-normalisation branch, both domains, constant
image labels, and a 4 M-pixel class."""
import json

import numpy as np
import pytest
import torch

from aaclip import ops

pytestmark = pytest.mark.gpu


def _sk(pixel_label, image_label, pixel_preds, image_preds, domain):
    """The reference's metrics (forward_utils.py:241-271), unrounded."""
    from sklearn.metrics import average_precision_score, roc_auc_score
    if pixel_preds.max() != 1:
        pixel_preds = (pixel_preds - pixel_preds.min()) / (pixel_preds.max() - pixel_preds.min())
    if image_preds.max() != 1:
        image_preds = (image_preds - image_preds.min()) / (image_preds.max() - image_preds.min())
    pmax = pixel_preds.max(axis=(1, 2))
    image_preds = pmax if domain == "Medical" else pmax * 0.5 + image_preds * 0.5
    y, s = pixel_label.flatten(), pixel_preds.flatten()
    out = [roc_auc_score(y, s), average_precision_score(y, s)]
    if image_label.max() != image_label.min():
        out += [roc_auc_score(image_label, image_preds), average_precision_score(image_label, image_preds)]
    else:
        out += [0.0, 0.0]
    return out


def _dev_metrics(dev, masks, labels, pp, ip, domain):
    t = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (pp, masks, ip, labels)]
    return ops.metrics_eval(t[0], t[1], t[2], t[3], medical=(domain == "Medical"))


def _case(seed, N, S, levels=None, frac=0.08, neg=False, max_one=False):
    r = np.random.default_rng(seed)
    masks = (r.random((N, 1, S, S)) < frac).astype(np.float32)
    pp = r.standard_normal((N, S, S)).astype(np.float32) + 1.5 * masks[:, 0]
    if levels:  # heavy ties
        pp = np.round(pp * levels) / levels
    if not neg:
        pp = pp - pp.min() + np.float32(0.25)
    if max_one:
        pp = (pp / pp.max()).astype(np.float32)
        pp[0, 0, 0] = np.float32(1.0)
    ip = r.random(N).astype(np.float32)
    labels = (masks.reshape(N, -1).max(1) > 0).astype(np.int64)
    labels[0], labels[-1] = 0, 1
    return masks, labels, pp.astype(np.float32), ip


def test_metrics_golden(dev, golden):
    o = golden["ops"]
    ref = json.loads(str(o["met_result"]))
    for dom in ("Industrial", "Medical"):
        got = _dev_metrics(dev, o["met_masks"], o["met_labels"], o["met_pp"], o["met_ip"], dom)
        want = _sk(o["met_masks"], o["met_labels"], o["met_pp"].copy(), o["met_ip"].copy(), dom)
        assert np.allclose(got, want, rtol=0, atol=1e-9), (dom, got, want)
        keys = ("pixel AUC", "pixel AP", "image AUC", "image AP")
        assert [round(v, 4) * 100 for v in got] == pytest.approx([ref[dom][k] for k in keys], abs=1e-9)


@pytest.mark.parametrize("kw", [dict(), dict(levels=4), dict(levels=64, neg=True), dict(max_one=True),
                                dict(levels=2, frac=0.3), dict(neg=True, max_one=True)])
@pytest.mark.parametrize("domain", ["Industrial", "Medical"])
def test_metrics_vs_sklearn(dev, kw, domain):
    masks, labels, pp, ip = _case(3, 12, 48, **kw)
    got = _dev_metrics(dev, masks, labels, pp, ip, domain)
    want = _sk(masks, labels, pp.copy(), ip.copy(), domain)
    assert np.allclose(got, want, rtol=0, atol=1e-9), (got, want)


def test_metrics_constant_image_labels(dev):
    masks, labels, pp, ip = _case(5, 6, 32)
    labels[:] = 1
    got = _dev_metrics(dev, masks, labels, pp, ip, "Industrial")
    want = _sk(masks, labels, pp.copy(), ip.copy(), "Industrial")
    assert got[2:] == [0.0, 0.0] and np.allclose(got[:2], want[:2], rtol=0, atol=1e-9)


def test_metrics_single_pixel_class_raises(dev):
    from forward_utils import metrics_eval
    masks, labels, pp, ip = _case(6, 4, 16)
    masks[:] = 0
    with pytest.raises(ValueError):
        metrics_eval(masks, labels, pp, ip, "c", "Industrial")


def test_metrics_large_class(dev):
    """4 M pixels (~ a 36-image 336 px class), bf16-like ties from quantised maps."""
    masks, labels, pp, ip = _case(7, 36, 336, levels=512)
    got = _dev_metrics(dev, masks, labels, pp, ip, "Industrial")
    want = _sk(masks, labels, pp.copy(), ip.copy(), "Industrial")
    assert np.allclose(got, want, rtol=0, atol=1e-9), (got, want)


def test_forward_utils_metrics_device_tensors(dev):
    """The drop-in entry point on device tensors returns the reference's dict."""
    from forward_utils import metrics_eval
    masks, labels, pp, ip = _case(8, 10, 40, levels=16)
    r = metrics_eval(torch.from_numpy(masks).to(dev), torch.from_numpy(labels).to(dev),
                     torch.from_numpy(pp).to(dev), torch.from_numpy(ip).to(dev), "cls", "Industrial")
    want = _sk(masks, labels, pp.copy(), ip.copy(), "Industrial")
    assert r["class name"] == "cls"
    assert [r[k] for k in ("pixel AUC", "pixel AP", "image AUC", "image AP")] == \
        pytest.approx([round(v, 4) * 100 for v in want], abs=1e-9)


@pytest.mark.parametrize("N,S", [(4, 518), (3, 37), (5, 41), (1, 17)])
def test_metrics_ragged_pixel_counts(dev, N, S):
    """Pixel counts whose 4-byte arrays are not 256-B multiples (4 maps of 518^2: the
    reference's default size) — the workspace carve-up must still fit."""
    masks, labels, pp, ip = _case(N * S, N, S)
    if N == 1:
        labels[0] = 1
    got = _dev_metrics(dev, masks, labels, pp, ip, "Industrial")
    want = _sk(masks, labels, pp.copy(), ip.copy(), "Industrial")
    assert np.allclose(got, want, rtol=0, atol=1e-9), (got, want)


def test_forward_utils_metrics_golden(dev, golden):
    """The drop-in metrics_eval vs the reference's own metrics_eval output (golden_ops:
    forward_utils.py:233-280 run by tests/golden/make_golden.py), both domains."""
    import json
    from forward_utils import metrics_eval
    o = golden["ops"]
    ref = json.loads(str(o["met_result"]))
    for dom in ("Industrial", "Medical"):
        r = metrics_eval(o["met_masks"], o["met_labels"], o["met_pp"].copy(), o["met_ip"].copy(), "synthetic", dom)
        for k in ("pixel AUC", "pixel AP", "image AUC", "image AP"):
            assert r[k] == pytest.approx(ref[dom][k], abs=1e-9)
