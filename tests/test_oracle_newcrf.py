"""Pins the CPU oracle of the NewCRF decoder (oracle/newcrf.py) to reference goldens (CPU)."""
import numpy as np
import pytest
import torch

from oracle import newcrf as onc
from oracle.weights import fill_
from tests.golden.make_golden import NEWCRF_CASES

torch.set_num_threads(4)


def close_scaled(a, b, tol, what):
    a = a.detach().double().numpy() if torch.is_tensor(a) else np.asarray(a, dtype=np.float64)
    err = float(np.abs(a - b).max())
    assert err <= tol * float(np.abs(b).max()) + 1e-30, f"{what}: {err:.3g} vs {np.abs(b).max():.3g}"


def check_grads(module, g, prefix, rtol):
    names = list(g[f"{prefix}grad_names"])
    params = dict(module.named_parameters())
    assert sorted(names) == sorted(n for n, p in params.items() if p.grad is not None)
    got = np.array([float(params[n].grad.double().norm()) for n in names])
    np.testing.assert_allclose(got, g[f"{prefix}grad_norms"], rtol=rtol)
    for n in names:
        key = f"{prefix}grad::{n}"
        if key in g:
            close_scaled(params[n].grad, g[key], rtol, n)


@pytest.mark.parametrize("case", NEWCRF_CASES, ids=[c[0] for c in NEWCRF_CASES])
def test_newcrf_matches_reference(golden, case):
    tag, (ind, emb, vd, heads), _, _ = case
    g = golden("golden_newcrf.npz")
    m = fill_(onc.NewCRF(input_dim=ind, embed_dim=emb, v_dim=vd, window_size=7, num_heads=heads))
    assert list(m.state_dict().keys()) == list(g[f"{tag}::keys"])
    x = torch.from_numpy(g[f"{tag}::x"]).requires_grad_(True)
    v = torch.from_numpy(g[f"{tag}::v"]).requires_grad_(True)
    y = m(x, v)
    close_scaled(y, g[f"{tag}::y"], 1e-5, "y")
    y.backward(torch.from_numpy(g[f"{tag}::gy"]))
    close_scaled(x.grad, g[f"{tag}::gx"], 1e-4, "gx")
    close_scaled(v.grad, g[f"{tag}::gv"], 1e-4, "gv")
    check_grads(m, g, f"{tag}::", 1e-4)


def test_decoder_matches_reference(golden):
    g = golden("golden_newcrf.npz")
    dec = fill_(onc.Decoder())
    assert list(dec.state_dict().keys()) == list(g["dec::keys"])
    feats = [None] * 18
    for i in (4, 7, 13, 16, 17):
        feats[i] = torch.from_numpy(g[f"dec::feat{i}"]).requires_grad_(True)
    y = dec(feats)
    close_scaled(y, g["dec::y"], 1e-5, "decoder depth")
    y.backward(torch.from_numpy(g["dec::gy"]))
    for i in (4, 7, 13, 16, 17):
        close_scaled(feats[i].grad, g[f"dec::gfeat{i}"], 1e-4, f"gfeat{i}")
    check_grads(dec, g, "dec::", 1e-4)


def test_shift_mask_regions():
    m = onc.shift_mask(14, 21, 7, 3)
    assert m.shape == (6, 49, 49)
    assert float(m[0].abs().max()) == 0.0          # interior window: one region
    assert float((m[-1] == -100).float().mean()) > 0.5  # corner window: 4 regions
