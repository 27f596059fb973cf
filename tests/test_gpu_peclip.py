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


def _prof_count(labels, fn):
    """Launches of the given GEMM variant labels while fn() runs (the library's live profiler)."""
    import ctypes
    from clipmi import _lib
    L = _lib.lib()
    L.clipmi_prof_arm.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.clipmi_prof_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double)]
    cap = 4096
    _lib.check(L.clipmi_prof_arm(",".join(labels).encode(), cap), "prof_arm")
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        L.clipmi_prof_disarm()
    ms, fl = (ctypes.c_float * cap)(), (ctypes.c_double * cap)()
    return L.clipmi_prof_read(cap, ms, fl)


@pytest.mark.parametrize("D,heads,B,N", [(192, 4, 5, 33), (128, 4, 3, 50), (320, 4, 2, 17), (96, 2, 3, 11)])
def test_general_head_width_batched_matches_torch(D, heads, B, N):
    """head_dim 48 / 32 / 80 / 48 (ContextAdapter with num_heads that do not give 64; D = 320 and 96 take
    the any-width LayerNorm kernels, D = 96 is the reference's own init-test width): the strided-batched
    fp32 path (clipmi_gemm_batched + row softmax over all B * H * N rows) vs PyTorch's own
    nn.MultiheadAttention + nn.LayerNorm in fp32 with the same parameters (output, input gradient,
    every parameter gradient: max |diff| / max |ref| < 2e-4), and its GEMM launch count does not grow
    with B * H: the same number of launches at batch B and batch 1."""
    from clipmi import peclip
    torch.manual_seed(0)
    mod = peclip.ContextAdapter(D, heads, device="cuda", precision="fp32")
    assert mod.attention_precision == "fp32" and mod.head_dim != 64
    ref_attn = torch.nn.MultiheadAttention(D, heads, batch_first=True).cuda()
    ref_ln = torch.nn.LayerNorm(D).cuda()
    sd = mod.state_dict()
    with torch.no_grad():
        ref_attn.in_proj_weight.copy_(sd["mhsa.in_proj_weight"])
        ref_attn.in_proj_bias.copy_(sd["mhsa.in_proj_bias"])
        ref_attn.out_proj.weight.copy_(sd["mhsa.out_proj.weight"])
        ref_attn.out_proj.bias.copy_(sd["mhsa.out_proj.bias"])
        ref_ln.weight.copy_(torch.linspace(0.5, 1.5, D))
        ref_ln.bias.copy_(torch.linspace(-0.1, 0.1, D))
        sd["layer_norm.weight"], sd["layer_norm.bias"] = ref_ln.weight.detach().cpu(), ref_ln.bias.detach().cpu()
    mod.load_state_dict({k: v.cpu() for k, v in sd.items()})
    x = torch.randn(B, N, D, device="cuda")
    gy = torch.randn(B, N, D, device="cuda")
    xa, xr = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya = mod(xa)
    ya.backward(gy)
    yr = ref_ln(ref_attn(xr, xr, xr, need_weights=False)[0] + xr)
    yr.backward(gy)
    torch.cuda.synchronize()

    def rel(a, b):
        return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))
    assert rel(ya, yr) < 2e-4 and rel(xa.grad, xr.grad) < 2e-4
    pairs = {"mhsa.in_proj_weight": ref_attn.in_proj_weight, "mhsa.in_proj_bias": ref_attn.in_proj_bias,
             "mhsa.out_proj.weight": ref_attn.out_proj.weight, "mhsa.out_proj.bias": ref_attn.out_proj.bias,
             "layer_norm.weight": ref_ln.weight, "layer_norm.bias": ref_ln.bias}
    got = dict(mod.named_parameters())
    for k, rp in pairs.items():
        assert rel(got[k].grad, rp.grad) < 2e-4, k

    def step(bb):
        xx = torch.randn(bb, N, D, device="cuda", requires_grad=True)
        mod(xx).backward(torch.randn(bb, N, D, device="cuda"))
    labels = ["gemm_f32_batched", "gemm_f32"]
    assert _prof_count(labels, lambda: step(B)) == _prof_count(labels, lambda: step(1))
    assert _prof_count(["gemm_f32_batched"], lambda: step(B)) == 6  # scores, context; dP, dQ, dK, dV
