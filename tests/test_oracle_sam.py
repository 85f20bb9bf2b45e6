"""Pins the CPU oracle of the SAM decoder (oracle/sam.py) to reference goldens (CPU)."""
import pytest
import torch

from oracle import sam as osam
from oracle.weights import fill_
from tests.golden.make_golden import SAM_CASES
from tests.test_oracle_newcrf import check_grads, close_scaled

torch.set_num_threads(4)


@pytest.mark.parametrize("case", SAM_CASES, ids=[c[0] for c in SAM_CASES])
def test_sam_matches_reference(golden, case):
    tag, (ind, emb, vd, heads), _, _ = case
    g = golden("golden_sam.npz")
    m = fill_(osam.SAM(input_dim=ind, embed_dim=emb, v_dim=vd, window_size=7, num_heads=heads))
    assert list(m.state_dict().keys()) == list(g[f"{tag}::keys"])
    e = torch.from_numpy(g[f"{tag}::e"]).requires_grad_(True)
    q = torch.from_numpy(g[f"{tag}::q"]).requires_grad_(True)
    y = m(e, q)
    close_scaled(y, g[f"{tag}::y"], 1e-5, "y")
    y.backward(torch.from_numpy(g[f"{tag}::gy"]))
    close_scaled(e.grad, g[f"{tag}::ge"], 1e-4, "ge")
    close_scaled(q.grad, g[f"{tag}::gq"], 1e-4, "gq")
    check_grads(m, g, f"{tag}::", 1e-4)


def test_sam_decoder_matches_reference(golden):
    g = golden("golden_sam.npz")
    dec = fill_(osam.Decoder())
    assert list(dec.state_dict().keys()) == list(g["dec::keys"])
    feats = [None] * 18
    for i in (4, 7, 13, 16, 17):
        feats[i] = torch.from_numpy(g[f"dec::feat{i}"]).requires_grad_(True)
    y = dec(feats)
    close_scaled(y, g["dec::y"], 1e-5, "decoder depth")
    y.backward(torch.from_numpy(g["dec::gy"]))
    for i in (4, 7, 13, 16, 17):
        close_scaled(feats[i].grad, g[f"dec::gfeat{i}"], 1e-4, f"gfeat{i}")
    # 96 parameter-gradient norms; fp32 summation order differs from the reference's
    # windowed copies (one small norm sits at 1.1e-4 relative)
    check_grads(dec, g, "dec::", 3e-4)


def test_sam_mirror_keys_match_reference(golden):
    """The product module tree (HIP path) has the reference's state_dict keys (CPU construct only)."""
    from monocular_depth_estimation_amd.model_mobileV3_large_SAM import Decoder, PTModel
    g = golden("golden_sam.npz")
    assert list(Decoder().state_dict().keys()) == list(g["dec::keys"])
    m = PTModel()
    assert not any(p.requires_grad for p in m.Unet[0].parameters())  # frozen backbone (:167-169)
