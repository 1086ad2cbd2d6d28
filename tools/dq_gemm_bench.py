"""Go / no-go for the attention dQ as a batched GEMM over a stored dS^T (decoder shape
B=32, H=2, T=977, dh=192): dQ[q][d] = sum_k dS^T[k][q] K[k][d] per (b, h), bf16, written into
the dQKV rows as the fused dQ kernel does.  Prints us per call and TF/s."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def main():
    from fastspeech2 import ops, _native
    _native.load()
    B, H, T, dh = 32, 2, 977, 192
    D = H * dh
    for ldst in (1024, 984):
        dST = (torch.randn(B * H, T, ldst, device="cuda") * 0.1).to(torch.bfloat16)
        QKV = torch.randn(B * T, 3 * D, device="cuda").to(torch.bfloat16)
        dQKV = torch.zeros(B * T, 3 * D, device="cuda", dtype=torch.bfloat16)
        T8 = (T + 7) // 8 * 8
        fn = lambda: ops.gemm(T8, dh, T8, dST, ldst, QKV[:, D:], 3 * D, dQKV, 3 * D, dt=1,
                              a_kmajor=0, b_kmajor=0, kvalid=T, mvalid=T, batch=B * H,
                              batch_div=H, strides=(H * T * ldst, T * ldst, T * 3 * D, dh,
                                                    T * 3 * D, dh, 0, 0))
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            fn()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 20 * 1e3
        fl = 2.0 * B * H * T * T * dh
        # check one (b, h) against torch
        z, bb, hh = 3, 1, 1
        ref = dST[z, :, :T].float().t() @ QKV[bb * T:(bb + 1) * T, D + hh * dh:D + (hh + 1) * dh].float()
        got = dQKV[bb * T:(bb + 1) * T, hh * dh:(hh + 1) * dh].float()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        print(f"ldst={ldst}: {us:.1f} us  {fl / us / 1e6:.0f} TF/s  rel err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
