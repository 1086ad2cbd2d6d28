"""Locate wrong outputs of the conv_mode 6 GEMM: per split plane against a torch reference of
that plane's K range, reporting the wrong (row-tile, col-tile) blocks and row / column sets."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def run(Bn, T, O, Cin, KW, S, seed=0):
    from fastspeech2 import ops
    torch.manual_seed(seed)
    P = (KW - 1) // 2
    M = Bn * T
    X = torch.randn(Bn, T, Cin, device="cuda").to(torch.bfloat16)
    G = torch.randn(M, O, device="cuda").to(torch.bfloat16)
    Kp = ops.round_up(Bn * (T + 2 * P), 64 * S)
    gy = torch.zeros(O * Kp + 128, device="cuda").to(torch.bfloat16)
    gx = torch.zeros(Cin * Kp + 128, device="cuda").to(torch.bfloat16)
    dYT, XT = gy[64:64 + O * Kp], gx[64:64 + Cin * Kp]
    ops.pad_transpose(G, O, Bn, T, O, P, 0, dYT, Kp, Kp, dt=1)
    ops.pad_transpose(X, Cin, Bn, T, Cin, P, 1, XT, Kp, Kp, dt=1)
    stride = O * KW * Cin
    ws = torch.full((S, O, KW * Cin), float("nan"), device="cuda")
    ops.gemm(O, KW * Cin, Kp, dYT, Kp, XT, Kp, ws, KW * Cin, dt=1, conv=(6, T, KW, Cin),
             c_fp32=1, split_k=S, split_stride=stride if S > 1 else 0)
    torch.cuda.synchronize()
    A = dYT.reshape(O, Kp).float()
    xg = gx.float()
    Bm = torch.stack([xg[64 + c * Kp + j - P: 64 + c * Kp + j - P + Kp] for j in range(KW)
                      for c in range(Cin)])      # [KW*Cin][Kp]
    kps = Kp // S
    bad_total = 0
    for s in range(S):
        ref = A[:, s * kps:(s + 1) * kps] @ Bm[:, s * kps:(s + 1) * kps].t()
        err = (ws[s] - ref).abs() > 1e-3 * ref.abs().max()
        nb = int(err.sum())
        bad_total += nb
        if nb:
            r, c = err.nonzero(as_tuple=True)
            tiles = sorted(set(zip((r // 256).tolist(), (c // 256).tolist())))
            print(f"  plane {s}: {nb} wrong; tiles {tiles[:12]}; rows {sorted(set((r % 256).tolist()))[:20]}"
                  f" cols {sorted(set((c % 256).tolist()))[:20]}", flush=True)
    print(f"B={Bn} T={T} O={O} C={Cin} KW={KW} S={S} Kp={Kp}: {bad_total} wrong", flush=True)


def main():
    from fastspeech2 import _native
    _native.load()
    for args in ((32, 977, 1536, 384, 9, 3), (32, 977, 1536, 384, 9, 3), (32, 200, 1536, 384, 9, 3),
                 (4, 77, 600, 72, 9, 1), (3, 130, 520, 128, 5, 2), (32, 977, 1536, 384, 9, 1)):
        run(*args)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def structured(Bn=4, T=77, O=600, Cin=72, KW=9, S=1):
    """A[m][k] = m + 1 and B image rows c = c + 1 over the valid columns: a wrong element's value
    names the (row, channel) pair it was computed from."""
    from fastspeech2 import ops
    P = (KW - 1) // 2
    Kp = ops.round_up(Bn * (T + 2 * P), 64 * S)
    gy = torch.zeros(O * Kp + 128, device="cuda").to(torch.bfloat16)
    gx = torch.zeros(Cin * Kp + 128, device="cuda").to(torch.bfloat16)
    n = 256
    A = (torch.arange(O, device="cuda").float() % 7 + 1)[:, None].expand(O, Kp).contiguous()
    A[:, n:] = 0
    Bv = (torch.arange(Cin, device="cuda").float() % 5 + 1)[:, None].expand(Cin, Kp).contiguous()
    gy[64:64 + O * Kp] = A.reshape(-1).to(torch.bfloat16)
    gx[64:64 + Cin * Kp] = Bv.reshape(-1).to(torch.bfloat16)
    dYT, XT = gy[64:64 + O * Kp], gx[64:64 + Cin * Kp]
    stride = O * KW * Cin
    ws = torch.full((S, O, KW * Cin), float("nan"), device="cuda")
    ops.gemm(O, KW * Cin, Kp, dYT, Kp, XT, Kp, ws, KW * Cin, dt=1, conv=(6, T, KW, Cin),
             c_fp32=1, split_k=S, split_stride=stride if S > 1 else 0)
    torch.cuda.synchronize()
    xg = gx.float()
    Bm = torch.stack([xg[64 + c * Kp + j - P: 64 + c * Kp + j - P + Kp] for j in range(KW)
                      for c in range(Cin)])
    ref = dYT.reshape(O, Kp).float() @ Bm.t()
    got = ws.sum(0)
    err = (got - ref).abs() > 1e-3 * ref.abs().max()
    r, c = err.nonzero(as_tuple=True)
    print(f"structured: {int(err.sum())} wrong of {err.numel()}")
    for k in range(min(24, r.numel())):
        m_, n_ = int(r[k]), int(c[k])
        print(f"  m={m_} n={n_}: got {got[m_, n_].item():.1f} ref {ref[m_, n_].item():.1f} "
              f"(A row val {m_ % 7 + 1}, B chan val {(n_ % Cin) % 5 + 1}; got/(n*Aval) "
              f"{got[m_, n_].item() / n / (m_ % 7 + 1):.3f})")


def plain_long(M=10752, N=1536, K=16384):
    """the same persistent kernel without BT (K-major plain GEMM, fp32 out, 256-wide tiles)"""
    from fastspeech2 import ops
    torch.manual_seed(1)
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    W = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    C = torch.full((M, N), float("nan"), device="cuda")
    ops.gemm(M, N, K, A, K, W, K, C, N, dt=1, c_fp32=1)
    ref = A.float() @ W.float().t()
    err = (C - ref).abs() > 1e-3 * ref.abs().max()
    r, c = err.nonzero(as_tuple=True)
    print(f"plain long K={K}: {int(err.sum())} wrong; rows%16 {sorted(set((r % 16).tolist()))} "
          f"cols%4 {sorted(set((c % 4).tolist()))}", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1:
    from fastspeech2 import _native
    _native.load()
    structured()
    structured(KW=1)
    structured(Bn=4, T=77, O=600, Cin=72, KW=9, S=1) if False else None
    plain_long()
