"""Diagnostic: s_memtime cycles per loop segment of the 8-wave dK/dV kernel (experiments
library, FS2_ATTN_FLAGS=64) at the decoder shape.
Segments: 0 next-tile DMA issue + counted wait, 1 barrier A, 2 S / dP MFMAs (issue), 3 softmax
VALU + P / dS pack, 4 dV / dK loop, 5 end barrier; cycles per tile, averaged over the blocks,
for waves 0-3 and 4-7."""
import math
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def main():
    from fastspeech2 import ops, _native
    _native.load()
    B, H, dh, T = 32, 2, 192, int(os.environ.get("ATTN_T", "977"))
    D = H * dh
    g = torch.Generator().manual_seed(T)
    lens = sorted([T] + torch.randint(T // 2, T + 1, (B - 1,), generator=g).tolist(), reverse=True)
    qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
    kp = torch.zeros(B, T, dtype=torch.uint8, device="cuda")
    for b, L in enumerate(lens):
        kp[b, L:] = 1
    out = torch.empty(B * T, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H, T, device="cuda")
    dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)
    dqkv = torch.empty(B * T, 3 * D, device="cuda", dtype=torch.bfloat16)
    nblk = (T + 127) // 128 * B * H
    base = int(ops.attn_ws(B, H, T))
    ws = torch.zeros(base + nblk * 8 * 32, device="cuda")
    sc = 1.0 / math.sqrt(dh)
    for p in [float(x) for x in os.environ.get("ATTN_P", "0,0.1").split(",")]:
        ops.attn_fwd(qkv, 3 * D, kp, B, H, T, dh, sc, p, 1, 2, out, D, lse, dt=1)
        for _ in range(3):
            ops.attn_bwd(qkv, 3 * D, kp, out, D, dout, D, lse, B, H, T, dh, sc, p, 1, 2,
                         dqkv, 3 * D, dt=1, ws=ws)
        torch.cuda.synchronize()
        st = ws[base:].view(torch.int64).view(nblk, 8, 16).cpu()
        nt = st[:, :, 6].double().clamp(min=1)
        per = st[:, :, :6].double() / nt[:, :, None]
        for grp, sl in (("waves 0-3", slice(0, 4)), ("waves 4-7", slice(4, 8))):
            m = per[:, sl].mean(dim=(0, 1))
            pro = st[:, sl, 7].double().mean().item()
            epi = st[:, sl, 8].double().mean().item()
            tot = (st[:, sl, 10] - st[:, sl, 9]).double().mean().item()
            print(f"p={p} {grp}: " + "  ".join(f"s{i} {m[i]:6.0f}" for i in range(6)) +
                  f"  loop {m.sum():6.0f}/tile; prologue {pro:7.0f} epilogue {epi:7.0f} "
                  f"block {tot:8.0f} cycles, {nt.mean().item():.1f} tiles", flush=True)
        span = (st[:, :, 10].max() - st[:, :, 9].min()).item()
        print(f"p={p}: kernel span {span} cycles (first entry to last end)", flush=True)


if __name__ == "__main__":
    main()
