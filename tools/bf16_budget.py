"""bf16 error budget of the bench path, by emulation on the fp32 oracle (CPU).

The bf16 engine stores every activation in bf16 and feeds bf16 operands to fp32-accumulating
MFMAs.  This script re-runs the oracle forward (oracle/fs2_oracle.py, eval, the B = 32 batch of
tests/test_gpu_fullsize.py) with bf16 rounding inserted at one class of storage sites at a time
and reports each class's contribution to the mel / PostNet error against the plain fp32 oracle
(mel L1 = mean |a - b| / mean |b|, as the parity test):

  weights    GEMM weight images (linear, conv, attention in / out projections)
  gemm_out   GEMM outputs stored in bf16 (QKV, attention context, projections, FFN hidden and
             output, predictor convs, concat projection, mel linear, PostNet convs)
  residual   the residual stream: LayerNorm outputs (encoder / decoder / predictors), the
             encoder and decoder inputs
  attn_p     attention probabilities (packed to bf16 for the P V MFMA)
  postnet    PostNet LayerNorm outputs (before tanh)
  gemm_in    GEMM input operands only (the MFMA operand rounding by itself: with an fp32
             residual stream the LayerNorm outputs would still enter the GEMMs in bf16)
  all        every site together -- compare with the GPU's observed bf16 error
             (profiles/*parity_observed.json: fullsize_fwd_b32_config3_bf16)

Usage: python tools/bf16_budget.py [out.json]     (~2 min on 8 cores; test infrastructure)
"""
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SITES = ("weights", "gemm_out", "residual", "attn_p", "postnet")
EXTRA = ("gemm_in",)
ON = set()


def rb(x, site):
    return x.to(torch.bfloat16).float() if site in ON else x


def mha_forward(self, q, k, v, attn_mask=None, key_padding_mask=None):
    """torch nn.MultiheadAttention (self-attention, eval) written out so the QKV, P and context
    storage can be rounded; equals the module's output to fp32 rounding (checked below)"""
    att = self.att
    B, T, D = q.shape
    H = att.num_heads
    dh = D // H
    qkv = rb(F.linear(rb(q, "gemm_in"), att.in_proj_weight, att.in_proj_bias), "gemm_out")
    Q, K, V = qkv.split(D, -1)

    def heads(t):   # torch's (T, B*H, dh) head split, index b * H + h
        return t.reshape(B, T, H, dh).permute(0, 2, 1, 3).reshape(B * H, T, dh)
    Q, K, V = heads(Q) * math.sqrt(1.0 / dh), heads(K), heads(V)
    S = torch.bmm(Q, K.transpose(1, 2))
    mask = key_padding_mask.view(B, 1, 1, T).expand(B, H, 1, T).reshape(B * H, 1, T)
    if attn_mask is not None:
        mask = mask | attn_mask
    P = rb(torch.softmax(S.masked_fill(mask, float("-inf")), -1), "attn_p")
    O = torch.bmm(P, V).reshape(B, H, T, dh).permute(0, 2, 1, 3).reshape(B, T, D)
    O = rb(rb(O, "gemm_out"), "gemm_in")
    return rb(F.linear(O, att.out_proj.weight, att.out_proj.bias), "gemm_out"), None


def build(kw, seed):
    from oracle import fs2_oracle as fo
    torch.manual_seed(seed)
    o = fo.FastSpeech2Oracle(**kw, n_speakers=4).eval()
    return o


def instrument(o):
    from oracle import fs2_oracle as fo
    import types
    for name, mod in o.named_modules():
        if isinstance(mod, fo.SBMultiheadAttention):
            mod.forward = types.MethodType(mha_forward, mod)
        elif isinstance(mod, (torch.nn.Linear, torch.nn.Conv1d)):
            mod.register_forward_hook(lambda m, i, out: rb(out, "gemm_out"))
            mod.register_forward_pre_hook(lambda m, i: (rb(i[0], "gemm_in"),) + tuple(i[1:]))
        elif isinstance(mod, torch.nn.LayerNorm):
            site = "postnet" if name.startswith("postnet.") else "residual"
            mod.register_forward_hook(lambda m, i, out, s=site: rb(out, s))
        elif isinstance(mod, fo.SBTransformerEncoder):
            mod.register_forward_pre_hook(
                lambda m, args, kwargs: ((rb(args[0], "residual"),) + tuple(args[1:]), kwargs),
                with_kwargs=True)


def round_weights(o):
    with torch.no_grad():
        for name, p in o.named_parameters():
            if name.endswith("weight") and p.dim() >= 2 and "Embedding" not in name:
                p.copy_(p.to(torch.bfloat16).float())


def main(out=None):
    from fastspeech2 import load_config
    from fastspeech2.synthetic import make_batch, as_tuple
    torch.set_num_threads(min(32, os.cpu_count() or 1))
    cfg = load_config()
    kw = cfg["model"]["fastspeech2"]
    b = make_batch(B=32, seed=11)       # tests/test_gpu_fullsize.py b32_config3
    bt, inten = as_tuple(b)
    args = (bt[0], bt[1], bt[6], bt[4], bt[5])

    def run(sites):
        ON.clear()
        ON.update(sites)
        o = build(kw, 4)
        instrument(o)
        if "weights" in sites:
            round_weights(o)
        t0 = time.time()
        with torch.no_grad():
            po = o(*args, intensity=inten)
        return po, time.time() - t0

    ref, t_ref = run(())
    # the hand-written attention equals torch's module (no rounding on)
    from oracle import fs2_oracle as fo
    with torch.no_grad():
        plain = build(kw, 4)(*args, intensity=inten)
    attn_check = max(((a - r).abs().max() / r.abs().max()).item()
                     for a, r in zip(ref[:2], plain[:2]))
    res = {"batch": "make_batch(B=32, seed=11), T_mel,max %d, eval, oracle seed 4" % bt[3].shape[1],
           "metric": "mel_l1 = mean|a-b| / mean|b| (test_gpu_fullsize._observe); *_maxrel = max|a-b| / max|b|",
           "manual_attention_vs_torch_maxrel": attn_check, "sites": {}}
    combos = {s: (s,) for s in SITES + EXTRA}
    combos["all"] = SITES + EXTRA
    # what an fp32 residual stream would leave: every other site, the LayerNorm outputs still
    # rounded where they enter a GEMM
    combos["all_but_residual"] = tuple(x for x in SITES + EXTRA if x != "residual")
    combos["all_but_residual_weights"] = tuple(x for x in SITES + EXTRA if x not in ("residual", "weights"))
    for s, sites in combos.items():
        po, dt = run(sites)
        r = {}
        for i, nm in ((0, "mel"), (1, "postnet")):
            a, ref_i = po[i], ref[i]
            r[nm + "_l1"] = ((a - ref_i).abs().mean() / ref_i.abs().mean()).item()
            r[nm + "_maxrel"] = ((a - ref_i).abs().max() / ref_i.abs().max()).item()
        for i, nm in ((2, "log_dur"), (3, "pitch"), (5, "energy")):
            r[nm + "_maxrel"] = ((po[i] - ref[i]).abs().max() / ref[i].abs().max()).item()
        res["sites"][s] = r
        print(f"{s:26s} mel L1 {r['mel_l1']:.2e}  mel maxrel {r['mel_maxrel']:.2e}  "
              f"postnet L1 {r['postnet_l1']:.2e}  ({dt:.1f} s)", flush=True)
    if out:
        json.dump(res, open(out, "w"), indent=1)
    return res


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
