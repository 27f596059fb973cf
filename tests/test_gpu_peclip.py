"""adapter/peclip.py's modules on libclipmi (clipmi.peclip) against the reference's own run
(tests/golden/peclip.npz, tools/gen_goldens.py gen_peclip): ContextAdapter / SharedAdapter =
layer_norm(mhsa(x, x, x) + x) through the fused in-projection GEMM, the flash attention kernels
(head_dim 64) or the per-head GEMM + row-softmax path (head_dim 48), the out-projection GEMM with
bias + residual and the LayerNorm kernel; TextualAdapter through towers.AdapterFn."""
import numpy as np
import pytest
import torch

from clipmi import synth

pytestmark = pytest.mark.gpu

CASES = [("ctx_n7", "ContextAdapter", 128, 2, (2, 7)), ("ctx_n197", "ContextAdapter", 128, 2, (2, 197)),
         ("shared_hd48", "SharedAdapter", 192, 4, (2, 9)), ("ctx_unbatched", "ContextAdapter", 128, 2, (11,))]


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-6))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("tag,cls,D,heads,shape", CASES)
def test_mhsa_adapter_matches_reference(golden, precision, tag, cls, D, heads, shape):
    """Output, input gradient and every parameter gradient vs the reference module.  Bounds: fp32
    max |diff| / max |ref| < 2e-4 (fp32 GEMMs and attention, different summation order); bf16
    (bf16 operands, fp32 accumulation) < 5e-2 on activations and 0.1 on parameter gradients, plus
    cosine > 0.999 per tensor.  head_dim 48 computes in fp32 in both modes (the general path;
    bf16 rounds only its input)."""
    from clipmi import peclip
    g = golden("peclip.npz")
    mod = getattr(peclip, cls)(D, heads, device="cuda", precision=precision)
    mod.load_state_dict({k: torch.from_numpy(v) for k, v in synth.mhsa_adapter_state_dict(D, 13, tag).items()})
    dtype = torch.bfloat16 if precision == "bf16" else torch.float32
    x = torch.from_numpy(synth.normal(shape + (D,), 13, f"{tag}/x")).cuda().to(dtype).requires_grad_(True)
    gy = torch.from_numpy(synth.normal(shape + (D,), 13, f"{tag}/gy")).cuda()
    y = mod(x)
    assert y.shape == x.shape and y.dtype == dtype
    y.float().backward(gy)
    torch.cuda.synchronize()
    exact = precision == "fp32"
    tol, gtol = (2e-4, 2e-4) if exact else (5e-2, 0.1)
    got = {"y": y.detach().float().cpu().numpy(), "gx": x.grad.float().cpu().numpy()}
    got.update({f"g/{k}": p.grad.cpu().numpy() for k, p in mod.named_parameters()})
    for k, v in got.items():
        ref = g[f"{tag}_{k}"]
        assert _rel(v, ref) < (gtol if k.startswith("g/") else tol), k
        cos = float((v * ref).sum() / (np.linalg.norm(v) * np.linalg.norm(ref) + 1e-30))
        assert cos > 0.999, (k, cos)


def test_mhsa_adapter_eval_no_grad_and_accumulation(golden):
    """Under torch.no_grad nothing is saved and the output is unchanged; two backward passes
    accumulate parameter gradients (AccumulateGrad semantics on the arena)."""
    from clipmi import peclip
    g = golden("peclip.npz")
    tag, D = "ctx_n7", 128
    mod = peclip.ContextAdapter(D, 2, device="cuda")
    mod.load_state_dict({k: torch.from_numpy(v) for k, v in synth.mhsa_adapter_state_dict(D, 13, tag).items()})
    x = torch.from_numpy(synth.normal((2, 7, D), 13, f"{tag}/x")).cuda()
    gy = torch.from_numpy(synth.normal((2, 7, D), 13, f"{tag}/gy")).cuda()
    with torch.no_grad():
        y0 = mod(x)
    assert _rel(y0.cpu().numpy(), g[f"{tag}_y"]) < 2e-4
    for _ in range(2):
        mod(x).backward(gy)
    torch.cuda.synchronize()
    w = mod.mhsa.in_proj_weight.grad.cpu().numpy()
    assert _rel(w, 2 * g[f"{tag}_g/mhsa.in_proj_weight"]) < 2e-4


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_textual_adapter_module_matches_reference(golden, precision):
    """clipmi.peclip.TextualAdapter (peclip.py:6-18) with adapters.npz's textual weights."""
    from clipmi import peclip
    g = golden("adapters.npz")
    D = 512
    mod = peclip.TextualAdapter(D, 256, device="cuda", precision=precision)
    sd = synth.adapter_state_dict(D, 256, 7, "textual_adapter", ln=False)
    mod.load_state_dict({k.replace("down_project", "down_proj").replace("up_project", "up_proj"): torch.from_numpy(v)
                         for k, v in sd.items()})
    x = torch.from_numpy(synth.normal((2, 5, D), 7, "textual/x")).cuda().requires_grad_(True)
    gy = torch.from_numpy(synth.normal((2, 5, D), 7, "textual/gy")).cuda()
    y = mod(x)
    assert y.dtype == torch.float32
    y.backward(gy)
    torch.cuda.synchronize()
    tol = 1e-4 if precision == "fp32" else 5e-2
    assert _rel(y.detach().cpu().numpy(), g["textual_y"]) < tol
    assert _rel(x.grad.cpu().numpy(), g["textual_gx"]) < tol
    for k, p in mod.named_parameters():
        assert _rel(p.grad.cpu().numpy(), g[f"textual_g/{k}"]) < (tol if precision == "fp32" else 0.1), k
