"""Fused attention fwd / bwd timing at the bench's decoder (T=977) and encoder (T=200) shapes,
B=32, H=2, dh=192, with and without probability dropout."""
import math
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def main():
    from fastspeech2 import ops, _native
    _native.load()
    B, H, dh = 32, 2, 192
    D = H * dh
    # ATTN_T / ATTN_P / ATTN_N: restrict to one shape / dropout and n timed calls (PMC passes)
    Ts = [int(os.environ["ATTN_T"])] if os.environ.get("ATTN_T") else [977, 200]
    ps = [float(os.environ["ATTN_P"])] if os.environ.get("ATTN_P") else [0.0, 0.1]
    nrep = int(os.environ.get("ATTN_N", "20"))
    for T in Ts:
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
        ws = torch.empty(int(ops.attn_ws(B, H, T)), device="cuda")
        sc = 1.0 / math.sqrt(dh)
        for p in ps:
            f = lambda: ops.attn_fwd(qkv, 3 * D, kp, B, H, T, dh, sc, p, 1, 2, out, D, lse, dt=1)
            bw = lambda: ops.attn_bwd(qkv, 3 * D, kp, out, D, dout, D, lse, B, H, T, dh, sc, p, 1, 2,
                                      dqkv, 3 * D, dt=1, ws=ws)
            res = []
            for fn in (f, bw):
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(nrep):
                    fn()
                b.record()
                torch.cuda.synchronize()
                res.append(a.elapsed_time(b) / nrep * 1e3)
            fl = 4.0 * B * T * T * D
            print(f"T={T} p={p}: fwd {res[0]:7.1f} us ({fl / res[0] / 1e6:6.1f} TF/s)  "
                  f"bwd {res[1]:7.1f} us ({2.5 * fl / res[1] / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
