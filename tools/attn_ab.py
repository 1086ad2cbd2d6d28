"""Save the fused attention forward / backward outputs at the decoder bench shape (B=32, H=2,
dh=192, T=977, p=0.1) to an .npz, for bit-for-bit A/B comparison of two kernel variants run in
separate processes (FS2_HIP_LIB=...libfs2_hip_exp.so with an FS2_* switch).
Usage: attn_ab.py OUT.npz  |  attn_ab.py --cmp A.npz B.npz"""
import math
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import numpy as np  # noqa: E402


def main():
    if sys.argv[1] == "--cmp":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        for k in a.files:
            same = np.array_equal(a[k], b[k])
            print(f"{k}: {'bit-identical' if same else 'DIFFERENT'}"
                  + ("" if same else f" (max |d| {np.abs(a[k].astype(np.float64) - b[k]).max():.3e})"))
        return
    import torch
    from fastspeech2 import ops, _native
    _native.load()
    B, H, dh, T = 32, 2, 192, 977
    D = H * dh
    g = torch.Generator().manual_seed(5)
    lens = sorted([T] + torch.randint(T // 2, T + 1, (B - 1,), generator=g).tolist(), reverse=True)
    torch.manual_seed(5)
    qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
    kp = torch.zeros(B, T, dtype=torch.uint8, device="cuda")
    for b, L in enumerate(lens):
        kp[b, L:] = 1
    out = torch.empty(B * T, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H, T, device="cuda")
    dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)
    dqkv = torch.empty(B * T, 3 * D, device="cuda", dtype=torch.bfloat16)
    ws = torch.empty(int(ops.attn_ws(B, H, T)), device="cuda")
    sc = 1.0 / math.sqrt(dh)
    ops.attn_fwd(qkv, 3 * D, kp, B, H, T, dh, sc, 0.1, 7, 3, out, D, lse, dt=1)
    ops.attn_bwd(qkv, 3 * D, kp, out, D, dout, D, lse, B, H, T, dh, sc, 0.1, 7, 3, dqkv, 3 * D,
                 dt=1, ws=ws)
    torch.cuda.synchronize()
    np.savez(sys.argv[1], out=out.view(torch.int16).cpu().numpy(), lse=lse.cpu().numpy(),
             dqkv=dqkv.view(torch.int16).cpu().numpy())


if __name__ == "__main__":
    main()
