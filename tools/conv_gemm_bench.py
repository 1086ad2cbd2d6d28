"""The decoder FFN conv1 GEMMs in isolation (B=32, T=977, D=384, F=1536, k=9, bf16): implicit
reflect-conv forward, padded-domain data gradient (fp32 out, unsplit), weight gradient."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    from fastspeech2 import ops, _native
    _native.load()
    Bn, T, C, O, KW = 32, 977, 384, 1536, 9
    P = (KW - 1) // 2
    M, Mp = Bn * T, Bn * (T + 2 * P)
    X = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    Wf = (torch.randn(O, KW * C, device="cuda") * 0.05).to(torch.bfloat16)
    Wb = (torch.randn(C, KW * O, device="cuda") * 0.05).to(torch.bfloat16)
    G = torch.randn(M, O, device="cuda").to(torch.bfloat16)
    bias = torch.randn(O, device="cuda")
    Y = torch.empty(M, O, device="cuda", dtype=torch.bfloat16)
    Xpad = torch.empty(Mp, C, device="cuda")
    fl = 2.0 * M * O * KW * C
    u = t(lambda: ops.gemm(M, O, KW * C, X, C, Wf, KW * C, Y, O, dt=1, conv=(1, T, KW, C), bias=bias, relu=1))
    print(f"conv1 fwd   {u:7.1f} us {fl / u / 1e6:7.1f} TF/s", flush=True)
    u = t(lambda: ops.gemm(Mp, C, KW * O, G, O, Wb, KW * O, Xpad, C, dt=1, conv=(4, T, KW, O), c_fp32=1))
    print(f"conv1 dgrad {u:7.1f} us {fl / u / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
