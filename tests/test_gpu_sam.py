"""SAM cross-window attention decoder on MI355X vs reference goldens and the
CPU oracle.  Tolerances as the NewCRF tests: outputs 1e-4, gradients 1e-3
(scale-relative; fp32 MFMA products, different summation orders)."""
import numpy as np
import pytest
import torch

from oracle import sam as osam
from oracle.weights import fill_, seeded
from tests.golden.make_golden import SAM_CASES
from tests.test_gpu_newcrf import close_scaled

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")


@pytest.mark.parametrize("case", SAM_CASES, ids=[c[0] for c in SAM_CASES])
def test_sam_golden(golden, case):
    from monocular_depth_estimation_amd.SAM import SAM
    tag, (ind, emb, vd, heads), _, _ = case
    g = golden("golden_sam.npz")
    m = fill_(SAM(input_dim=ind, embed_dim=emb, v_dim=vd, window_size=7, num_heads=heads)).to(DEV)
    assert list(m.state_dict().keys()) == list(g[f"{tag}::keys"])
    e = torch.from_numpy(g[f"{tag}::e"]).to(DEV).requires_grad_(True)
    q = torch.from_numpy(g[f"{tag}::q"]).to(DEV).requires_grad_(True)
    y = m(e, q)
    close_scaled(y, g[f"{tag}::y"], 1e-4, "y")
    y.backward(torch.from_numpy(g[f"{tag}::gy"]).to(DEV))
    close_scaled(e.grad, g[f"{tag}::ge"], 1e-3, "ge")
    close_scaled(q.grad, g[f"{tag}::gq"], 1e-3, "gq")
    params = dict(m.named_parameters())
    names = list(g[f"{tag}::grad_names"])
    got = np.array([float(params[n].grad.double().norm()) for n in names])
    np.testing.assert_allclose(got, g[f"{tag}::grad_norms"], rtol=1e-3)
    for key in g:
        if key.startswith(f"{tag}::grad::"):
            n = key[len(f"{tag}::grad::"):]
            close_scaled(params[n].grad, g[key], 1e-3, n)


@pytest.mark.parametrize("b,h,w,emb,heads", [(2, 30, 40, 256, 8), (1, 15, 20, 1024, 32),
                                             (2, 7, 7, 128, 4)])
def test_sam_block_vs_oracle(b, h, w, emb, heads):
    """One SAMBLOCK at decoder-stage shapes (incl. padded windows) vs the oracle."""
    from monocular_depth_estimation_amd.SAM import SAMBLOCK
    ref = fill_(osam.SAMBLOCK(emb, heads, 7))
    hip = fill_(SAMBLOCK(emb, heads, emb, 7)).to(DEV)
    x = torch.from_numpy(seeded((b, h * w, emb), 11, -1, 1))
    v = torch.from_numpy(seeded((b, h * w, emb), 12, -1, 1))
    gy = torch.from_numpy(seeded((b, h * w, emb), 13, -1, 1))
    xr, vr = x.clone().requires_grad_(True), v.clone().requires_grad_(True)
    yr = ref(xr, vr, h, w)
    yr.backward(gy)
    xd, vd = x.to(DEV).requires_grad_(True), v.to(DEV).requires_grad_(True)
    yd, _, _ = hip(xd, vd, h, w)
    close_scaled(yd, yr, 1e-4, "y")
    yd.backward(gy.to(DEV))
    close_scaled(xd.grad, xr.grad, 1e-3, "gx")
    close_scaled(vd.grad, vr.grad, 1e-3, "gv")
    close_scaled(hip.attn.kv.bias.grad, ref.attn.kv.bias.grad, 1e-3, "kv bias (incl. padded v)")
    close_scaled(hip.attn.q.bias.grad, ref.attn.q.bias.grad, 1e-3, "q bias")


def test_sam_decoder_golden(golden):
    from monocular_depth_estimation_amd.model_mobileV3_large_SAM import Decoder
    g = golden("golden_sam.npz")
    dec = fill_(Decoder()).to(DEV)
    feats = [None] * 18
    for i in (4, 7, 13, 16, 17):
        feats[i] = torch.from_numpy(g[f"dec::feat{i}"]).to(DEV).requires_grad_(True)
    y = dec(feats)
    close_scaled(y, g["dec::y"], 1e-4, "decoder depth")
    y.backward(torch.from_numpy(g["dec::gy"]).to(DEV))
    for i in (4, 7, 13, 16, 17):
        close_scaled(feats[i].grad, g[f"dec::gfeat{i}"], 1e-3, f"gfeat{i}")
