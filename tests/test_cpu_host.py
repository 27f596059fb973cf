"""Host-side checks that need no GPU: the C-ABI library loads and exports every entry
point include/clipmi.h declares; parameter names/shapes match HF CLIPModel and the
reference adapter checkpoint; the trainer's error behaviour; the data-parallel
contrastive decomposition over a 2-rank gloo group."""
import json
import os
import re

import numpy as np
import pytest
import torch

from clipmi import config as C
from clipmi import synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(REPO, "include", "clipmi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(clipmi_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from clipmi import _lib
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert L.clipmi_version() >= 1


def test_library_built_from_these_sources():
    """Build provenance: the loaded libclipmi.so carries the sha256 of the sources it was compiled
    from (Makefile DIGEST_SRC), equal to the digest of the sources in this tree -- the same check
    _lib.lib() makes before any op runs, here or on a GPU box."""
    from clipmi import _lib
    assert _lib.build_digest() == _lib.source_digest()


def test_invalid_args_raise_without_gpu():
    """Argument validation runs on the host before any launch."""
    from clipmi import _lib
    from clipmi._lib import GemmDesc
    import ctypes
    d = GemmDesc()
    d.M, d.N, d.K = 16, 12, 64  # N % 8 != 0
    d.ab_dtype = d.c_dtype = 1
    st = _lib.lib().clipmi_gemm(None, ctypes.byref(d))
    assert st == -1 and b"N % 8" in _lib.lib().clipmi_last_error()
    with pytest.raises(ValueError):
        _lib.check(st, "clipmi_gemm")


def _gemm_desc(flags, **ptrs):
    from clipmi._lib import GemmDesc
    d = GemmDesc()
    d.M, d.N, d.K = 256, 256, 64
    d.ab_dtype = d.c_dtype = 1
    d.A, d.B, d.C = 4096, 8192, 12288  # never dereferenced: validation rejects before any launch
    d.lda = d.ldb = 64
    d.ldc = d.ldr = d.ldaux = 256
    d.alpha = 1.0
    d.flags = flags
    for k, v in ptrs.items():
        setattr(d, k, v)
    return d


@pytest.mark.parametrize("flag,operand", [
    ("EPI_DQGELU", "aux"), ("EPI_DGELU", "aux"), ("EPI_MUL_AUX", "aux"), ("EPI_STORE_PRE", "aux"),
    ("EPI_STORE_DACT", "aux"), ("EPI_RESID", "residual"), ("EPI_BIAS", "bias")])
def test_epilogue_flag_without_operand_is_rejected(flag, operand):
    """Every epilogue flag that reads or writes an operand returns CLIPMI_ERR_INVALID when that
    operand is missing, before any launch: a null aux with an aux-reading epilogue once faulted a
    GPU in a bench tool (csrc/gemm.hip clipmi_gemm validation)."""
    import ctypes
    from clipmi import _lib
    f = getattr(_lib, flag)
    if flag == "EPI_STORE_DACT":
        f |= _lib.EPI_QGELU
    ptrs = {"aux": 16384, "residual": 20480, "bias": 24576}
    ptrs[operand] = None
    d = _gemm_desc(f, **ptrs)
    st = _lib.lib().clipmi_gemm(None, ctypes.byref(d))
    assert st == -1, (flag, st)
    assert operand.encode()[:3] in _lib.lib().clipmi_last_error()


@pytest.mark.parametrize("case", ["D", "A", "ln_w", "saved", "ws"])
def test_adapter_bad_arguments_rejected(case):
    """clipmi_adapter_fwd / _bwd reject D or A not a multiple of 8 in bf16 (16-byte MFMA rows; fp32 takes any
    width, as nn.Linear does: test_gpu_kernels.test_adapter_fused_pooled_rows_matches_torch), ln without its
    weights, a missing activation buffer (act carries the bottleneck between the launches) and a short backward
    workspace with CLIPMI_ERR_INVALID before any launch (pointers here are never dereferenced)."""
    from clipmi import _lib
    from clipmi import towers as T  # noqa: F401  (declares the prototypes)
    L = _lib.lib()
    p = 4096
    R, D, A = 4, 512, 64
    if case == "ws":
        need = L.clipmi_adapter_bwd_ws(R, D, A)
        assert need >= (R * (D + A)) * 4  # dz + d_pre (fp32-sized) + the LN / column-sum scratch
        st = L.clipmi_adapter_bwd(None, 0, R, D, A, p, D, p, D, p, p, p, p, p, p, p, p, 1, p, D, *([None] * 6), p,
                                  need - 4)
    else:
        if case == "D":
            D = 510
        if case == "A":
            A = 60
        lnw = None if case == "ln_w" else p
        act = None if case == "saved" else p
        dt = _lib.BF16 if case in ("D", "A") else _lib.F32
        st = L.clipmi_adapter_fwd(None, dt, R, D, A, p, D, p, p, p, p, lnw, p, 1e-5, 1, p, D, p, act, p, p, p)
    assert st == -1, case


@pytest.mark.parametrize("combo", [("EPI_STORE_PRE", "EPI_STORE_DACT"), ("EPI_MUL_AUX", "EPI_RESID"),
                                   ("EPI_MUL_AUX", "EPI_BETA"), ("EPI_DQGELU", "EPI_STORE_PRE"),
                                   ("EPI_MUL_AUX", "EPI_DQGELU")])
def test_epilogue_flag_conflicts_are_rejected(combo):
    """Flag pairs that would give aux two roles, or feed one epilogue input stream to two
    operations, are rejected on the host (the kernels' static_asserts cover the compiled forms)."""
    import ctypes
    from clipmi import _lib
    f = _lib.EPI_QGELU
    for c in combo:
        f |= getattr(_lib, c)
    d = _gemm_desc(f, aux=16384, residual=20480, bias=24576)
    assert _lib.lib().clipmi_gemm(None, ctypes.byref(d)) == -1


def test_param_names_match_hf_clipmodel():
    from transformers import CLIPConfig, CLIPModel
    from clipmi.modules import CLIPParams
    cfg = C.resolve("tiny")
    hf = CLIPModel(CLIPConfig(**cfg.to_hf_dict()))
    ours = CLIPParams(cfg, "cpu", shadow=False)
    hs = {k: tuple(v.shape) for k, v in hf.state_dict().items() if not k.endswith("position_ids")}
    os_ = {k: tuple(v.shape) for k, v in ours.state_dict().items()}
    assert hs == os_
    # HF state dict loads into the arena-backed module and round-trips
    ours.load_state_dict(hf.state_dict(), strict=False)
    for k, v in hf.state_dict().items():
        if k in os_:
            assert torch.equal(ours.state_dict()[k], v)


def test_adapter_checkpoint_schema_matches_reference_fixture(golden):
    from clipmi.modules import AdapterParams
    schema = json.load(open(os.path.join(REPO, "tests", "golden", "test_adapter_schema.json")))
    for key, hidden in (("text_adapter", 512), ("vision_adapter", 768)):
        a = AdapterParams(hidden, 256, "cpu", shadow=False)
        assert {k: list(v.shape) for k, v in a.state_dict().items()} == schema[key]


def test_model_construction_and_checkpoint_roundtrip_cpu(tmp_path):
    from clipmi import CLIPWithAdapters
    m = CLIPWithAdapters("tiny", use_shared_adapters=False, device="cpu")
    assert all(not p.requires_grad for p in m.clip.parameters())
    assert all(p.requires_grad for n, p in m.named_parameters() if "adapter" in n)
    assert abs(m.clip.logit_scale.item() - C.LN100) < 1e-6
    path = str(tmp_path / "sub" / "ad.pt")
    m.save_adapter_weights(path)
    m2 = CLIPWithAdapters("tiny", use_shared_adapters=False, device="cpu", init_seed=5)
    assert not torch.equal(m2.text_adapter.down_project.weight, m.text_adapter.down_project.weight)
    m2.load_adapter_weights(path)
    assert torch.equal(m2.text_adapter.down_project.weight, m.text_adapter.down_project.weight)
    sd = torch.load(path, weights_only=True)
    assert set(sd) == {"text_adapter", "vision_adapter"}
    m3 = CLIPWithAdapters("tiny", use_vision_adapter=False, use_shared_adapters=False, device="cpu")
    with pytest.raises(ValueError, match="Vision adapter weights found"):
        m3.load_adapter_weights(path)
    with pytest.raises(FileNotFoundError):
        m3.load_adapter_weights(str(tmp_path / "nope.pt"))
    m4 = CLIPWithAdapters("tiny", use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                          device="cpu")
    with pytest.raises(ValueError, match="No adapters enabled"):
        m4.save_adapter_weights(path)


def test_trainer_empty_param_list_raises_like_torch():
    from clipmi import CLIPWithAdapters, CLIPAdapterTrainer
    m = CLIPWithAdapters("tiny", use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                         device="cpu")
    with pytest.raises(ValueError, match="empty parameter list"):
        CLIPAdapterTrainer(m, [], output_dir="/tmp/clipmi_t")


def test_arena_layout_fused_qkv_is_contiguous():
    from clipmi.modules import CLIPParams
    m = CLIPParams(C.resolve("tiny"), "cpu", shadow=False)
    a = m.arena
    q = a.offsets["vision_model.encoder.layers.1.self_attn.q_proj.weight"][0]
    v = a.offsets["vision_model.encoder.layers.1.self_attn.v_proj.weight"][0]
    D = 128
    assert v - q == 2 * D * D
    for name, (off, _, _) in a.offsets.items():
        assert off % 8 == 0, name
    # parameters are views of the arena: an in-place update shows in the flat buffer
    with torch.no_grad():
        m.vision_model.encoder.layers[1].self_attn.k_proj.weight.fill_(3.0)
    assert a.data[q + D * D: q + 2 * D * D].eq(3.0).all()


def test_flops_model_matches_survey():
    assert abs(C.forward_flops_per_pair(C.resolve("B/16")) / 1e9 - 41.086) < 0.01
    assert abs(C.forward_flops_per_pair(C.resolve("B/32")) / 1e9 - 14.777) < 0.01
    assert abs(C.forward_flops_per_pair(C.resolve("L/14")) / 1e9 - 175.325) < 0.01


def test_synthetic_batch_sharding_is_consistent():
    cfg = C.resolve("tiny")
    full = synth.synthetic_batch(cfg, 6, seed=7)
    a = synth.synthetic_batch(cfg, 3, seed=7, start=0)
    b = synth.synthetic_batch(cfg, 3, seed=7, start=3)
    for k in full:
        assert np.array_equal(full[k], np.concatenate([a[k], b[k]]))
    ids, mask = full["input_ids"], full["attention_mask"]
    assert (ids[:, 0] == cfg.text_config.bos_token_id).all()
    L = mask.sum(1)
    assert ((L >= 5) & (L <= 77)).all()


def _dp_worker(rank, world, port, q):
    import torch.distributed as dist
    import torch.nn.functional as F
    from clipmi import towers as T
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    Bg, E = 8, 16
    tg = torch.randn(Bg, E, dtype=torch.float64)
    ig = torch.randn(Bg, E, dtype=torch.float64)
    s = torch.tensor(2.0, dtype=torch.float64)
    B = Bg // world
    tl = tg[rank * B:(rank + 1) * B].clone().requires_grad_(True)
    il = ig[rank * B:(rank + 1) * B].clone().requires_grad_(True)
    # the same decomposition ContrastiveFn runs, with its collective helpers
    th, ih = tl / tl.norm(dim=-1, keepdim=True), il / il.norm(dim=-1, keepdim=True)
    tall = T._gather(th.detach(), None, world)
    iall = T._gather(ih.detach(), None, world)
    lab = torch.arange(B) + rank * B
    lt = s.exp() * th @ iall.t()
    li = s.exp() * ih @ tall.t()
    loss = (F.cross_entropy(lt, lab, reduction="sum") + F.cross_entropy(li, lab, reduction="sum")) / (2 * Bg)
    loss.backward()
    # column-direction gradient terms: d loss / d (gathered features), reduce-scattered to owners
    tall_r = tall.clone().requires_grad_(True)
    iall_r = iall.clone().requires_grad_(True)
    l2 = (F.cross_entropy(s.exp() * th.detach() @ iall_r.t(), lab, reduction="sum")
          + F.cross_entropy(s.exp() * ih.detach() @ tall_r.t(), lab, reduction="sum")) / (2 * Bg)
    l2.backward()
    gt_extra = T._reduce_scatter(tall_r.grad, None, world)
    gi_extra = T._reduce_scatter(iall_r.grad, None, world)
    # chain the extra normalized-feature gradient through the local normalisation
    th2 = tl.detach().clone().requires_grad_(True)
    (th2 / th2.norm(dim=-1, keepdim=True)).backward(gt_extra)
    ih2 = il.detach().clone().requires_grad_(True)
    (ih2 / ih2.norm(dim=-1, keepdim=True)).backward(gi_extra)
    lsum = loss.detach().clone()
    dist.all_reduce(lsum)
    q.put((rank, lsum.item(), (tl.grad + th2.grad).numpy(), (il.grad + ih2.grad).numpy()))
    dist.destroy_process_group()


def test_data_parallel_contrastive_decomposition_gloo():
    """Sum over 2 ranks of the sharded loss == single-device loss; sharded feature grads ==
    single-device grads."""
    import torch.multiprocessing as mp
    import torch.nn.functional as F
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(60)
    torch.manual_seed(0)
    Bg, E = 8, 16
    tg = torch.randn(Bg, E, dtype=torch.float64, requires_grad=True)
    ig = torch.randn(Bg, E, dtype=torch.float64, requires_grad=True)
    s = torch.tensor(2.0, dtype=torch.float64)
    L = s.exp() * (tg / tg.norm(dim=-1, keepdim=True)) @ (ig / ig.norm(dim=-1, keepdim=True)).t()
    lab = torch.arange(Bg)
    ref = (F.cross_entropy(L, lab) + F.cross_entropy(L.t(), lab)) / 2
    ref.backward()
    for rank, lsum, gt, gi in res:
        assert abs(lsum - ref.item()) < 1e-12
        np.testing.assert_allclose(gt, tg.grad[rank * 4:(rank + 1) * 4].numpy(), atol=1e-12)
        np.testing.assert_allclose(gi, ig.grad[rank * 4:(rank + 1) * 4].numpy(), atol=1e-12)


def test_shared_adapter_state_dict_schema():
    """shared_adapters.* names/shapes equal SharedMHSAttentionAdapter's (adapter/clip_adapter.py:70-97:
    Linear text/image projections, nn.MultiheadAttention, 3 LayerNorms, Sequential MLP)."""
    import torch.nn as nn
    from clipmi import CLIPWithAdapters
    m = CLIPWithAdapters("tiny", use_shared_adapters=True, shared_adapter_layers=2, device="cpu")
    t, v = m.config.text_config.hidden_size, m.config.vision_config.hidden_size
    H = 512
    ref = nn.ModuleDict(dict(text_proj=nn.Linear(t, H), image_proj=nn.Linear(v, H),
                             cross_attn=nn.MultiheadAttention(H, 8, batch_first=True),
                             norm1=nn.LayerNorm(H), norm2=nn.LayerNorm(H), norm3=nn.LayerNorm(H),
                             mlp=nn.Sequential(nn.Linear(H, 4 * H), nn.GELU(), nn.Linear(4 * H, H), nn.Dropout(0.1))))
    want = {k: tuple(x.shape) for k, x in ref.state_dict().items()}
    got = {k: tuple(x.shape) for k, x in m.shared_adapters[1].state_dict().items()}
    assert got == want
    names = [n for n, _ in m.named_parameters() if "shared_adapters" in n]
    assert len(names) == 2 * len(want) and all("adapter" in n for n in names)
    assert len(m.arenas()) == 5


def _reducer_worker(rank, world, port, q):
    import torch.distributed as dist
    from clipmi.arena import Arena
    from clipmi.trainer import GradBucketReducer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a = Arena([("w0", (300,)), ("w1", (17, 9)), ("w2", (1000,))], "cpu", dtype_shadow=False)
    b = Arena([("v", (70,))], "cpu", dtype_shadow=False)
    g = torch.Generator().manual_seed(rank)
    a.grad.copy_(torch.randn(a.numel, generator=g))
    b.grad.copy_(torch.randn(b.numel, generator=g))
    r = GradBucketReducer([a, b], dist.group.WORLD)
    # two buckets reported out of order (as a chunked backward does), the rest left to finish()
    r.ready(a, a.offsets["w2"][0], 1000)
    r.ready(a, 64, 128)
    r.finish()
    q.put((rank, a.grad.numpy().copy(), b.grad.numpy().copy()))
    dist.destroy_process_group()


def test_grad_bucket_reducer_sums_every_element_once_gloo():
    """GradBucketReducer (SURVEY §8e bucketed, overlapped all-reduce): reported buckets plus the
    complement finish() reduces = exactly one all-reduce of every arena element."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_reducer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(60)
    from clipmi.arena import Arena
    want_a, want_b = 0, 0
    for rank in range(2):
        g = torch.Generator().manual_seed(rank)
        a = Arena([("w0", (300,)), ("w1", (17, 9)), ("w2", (1000,))], "cpu", dtype_shadow=False)
        b = Arena([("v", (70,))], "cpu", dtype_shadow=False)
        want_a = want_a + torch.randn(a.numel, generator=g)
        want_b = want_b + torch.randn(b.numel, generator=g)
    for rank, ga, gb in res:
        np.testing.assert_allclose(ga, want_a.numpy(), rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(gb, want_b.numpy(), rtol=1e-6, atol=1e-6)


def test_bench_self_launches_n_ranks():
    """`bench.py --gpus 2` with no torch.distributed environment starts 2 ranks itself (through
    torch.distributed.run, before any GPU call); --launch-check stops each rank before the GPU."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted((d["rank"], d["world"]) for d in lines) == [(0, 2), (1, 2)]


@pytest.mark.parametrize("tag,cls,args", [("context", "ContextAdapter", (128, 2)), ("shared", "SharedAdapter", (96, 2)),
                                          ("textual", "TextualAdapter", (64, 32))])
def test_peclip_modules_init_like_reference(golden, tag, cls, args):
    """clipmi.peclip's constructors draw their parameters from torch's generator in the order
    nn.Linear / nn.MultiheadAttention do (adapter/peclip.py:8-11, 26-29, 40-43): under the same
    manual_seed the state dict equals the reference module's (tests/golden/peclip.npz), key for key."""
    from clipmi import peclip
    g = golden("peclip.npz")
    torch.manual_seed(5)
    mod = getattr(peclip, cls)(*args, device="cpu")
    sd = mod.state_dict()
    ref = sorted(k[len(f"init_{tag}/"):] for k in g.files if k.startswith(f"init_{tag}/"))
    assert sorted(sd) == ref
    for k in ref:
        assert np.array_equal(sd[k].numpy(), g[f"init_{tag}/{k}"]), k


def test_peclip_argument_errors():
    """nn.MultiheadAttention's checks (num_heads must divide embed_dim; the input's last dimension)
    and the precision switch; no CPU fallback for the forward."""
    from clipmi import peclip
    with pytest.raises(AssertionError, match="divisible"):
        peclip.ContextAdapter(100, 3, device="cpu")
    with pytest.raises(ValueError, match="precision"):
        peclip.SharedAdapter(64, 1, device="cpu", precision="fp16")
    m = peclip.ContextAdapter(64, 1, device="cpu")
    with pytest.raises(AssertionError, match="embedding dimension of 64, but got 32"):
        m(torch.zeros(2, 3, 32))
    with pytest.raises(ValueError, match="no CPU fallback"):
        m(torch.zeros(2, 3, 64))
