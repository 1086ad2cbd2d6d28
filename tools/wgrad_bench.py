"""Where does the decoder FFN conv1 weight gradient lose to the forward? (B=32, T=977, bf16)
(a) the engine's call: implicit reflect conv on the MN-major B operand (conv mode 3), split-K
    slices + fixed-order sum;
(b) the same GEMM on a materialised im2col (plain MN-major B), same slices;
(c) both operands K-major (dY^T and im2col^T materialised), same slices.
Prints us per call and TF/s of the 331.9 GFLOP product (operand materialisation not timed)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def timed(fn, n=10):
    for _ in range(2):
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
    B, T, C, F, KW = 32, 977, 384, 1536, 9
    P = (KW - 1) // 2
    M = B * T
    bf = torch.bfloat16
    dY = (torch.randn(M, F, device="cuda") * 0.5).to(bf)
    X = (torch.randn(M, C, device="cuda") * 0.5).to(bf)
    Ncols = KW * C
    fl = 2.0 * M * F * Ncols
    ns = 3
    stride = F * Ncols
    ws = torch.empty(ns * stride, device="cuda")
    out = torch.zeros(F, Ncols, device="cuda")
    K = (M + 7) // 8 * 8

    def a():
        ops.gemm(F, Ncols, K, dY, F, X, C, ws, Ncols, dt=1, a_kmajor=0, b_kmajor=0,
                 conv=(3, T, KW, C), c_fp32=1, kvalid=M, nvalid=Ncols, split_k=ns,
                 split_stride=stride)
        ops.sum_slices(ws, ns, stride, stride, out, accumulate=1)
    print(f"(a) conv3 MN-major       {timed(a):7.1f} us  {fl / timed(a) / 1e6:6.0f} TF/s", flush=True)
    # im2col (reflect) materialised: Xcol[t][(j, c)]
    idx = torch.arange(T, device="cuda")
    cols = []
    for j in range(KW):
        src = idx + j - P
        src = torch.where(src < 0, -src, src)
        src = torch.where(src >= T, 2 * (T - 1) - src, src)
        cols.append(X.view(B, T, C)[:, src, :])
    Xcol = torch.cat(cols, dim=2).reshape(M, Ncols).contiguous()
    del cols

    def b():
        ops.gemm(F, Ncols, K, dY, F, Xcol, Ncols, ws, Ncols, dt=1, a_kmajor=0, b_kmajor=0,
                 c_fp32=1, kvalid=M, nvalid=Ncols, split_k=ns, split_stride=stride)
        ops.sum_slices(ws, ns, stride, stride, out, accumulate=1)
    print(f"(b) im2col MN-major      {timed(b):7.1f} us  {fl / timed(b) / 1e6:6.0f} TF/s", flush=True)
    dYt = torch.zeros(F, K, device="cuda", dtype=bf)
    dYt[:, :M] = dY.t()
    Xct = torch.zeros(Ncols, K, device="cuda", dtype=bf)
    Xct[:, :M] = Xcol.t()
    del Xcol

    def c():
        ops.gemm(F, Ncols, K, dYt, K, Xct, K, ws, Ncols, dt=1, a_kmajor=1, b_kmajor=1,
                 c_fp32=1, nvalid=Ncols, split_k=ns, split_stride=stride)
        ops.sum_slices(ws, ns, stride, stride, out, accumulate=1)
    print(f"(c) both K-major         {timed(c):7.1f} us  {fl / timed(c) / 1e6:6.0f} TF/s", flush=True)

    def e():   # A K-major (dY^T), B MN-major implicit reflect conv
        ops.gemm(F, Ncols, K, dYt, K, X, C, ws, Ncols, dt=1, a_kmajor=1, b_kmajor=0,
                 conv=(3, T, KW, C), c_fp32=1, kvalid=M, nvalid=Ncols, split_k=ns,
                 split_stride=stride)
        ops.sum_slices(ws, ns, stride, stride, out, accumulate=1)
    print(f"(e) A K-major, B conv3 MN-major {timed(e):7.1f} us  {fl / timed(e) / 1e6:6.0f} TF/s", flush=True)

    def f():   # A MN-major (dY), B K-major (im2col^T)
        ops.gemm(F, Ncols, K, dY, F, Xct, K, ws, Ncols, dt=1, a_kmajor=0, b_kmajor=1,
                 c_fp32=1, kvalid=M, nvalid=Ncols, split_k=ns, split_stride=stride)
        ops.sum_slices(ws, ns, stride, stride, out, accumulate=1)
    print(f"(f) A MN-major, B K-major       {timed(f):7.1f} us  {fl / timed(f) / 1e6:6.0f} TF/s", flush=True)

    def tr():  # the dY transpose itself (torch), for the cost side
        dYt[:, :M].copy_(dY.t())
    print(f"(t) dY^T by torch copy          {timed(tr):7.1f} us", flush=True)

    def c1():
        ops.gemm(F, Ncols, K, dYt, K, Xct, K, out, Ncols, dt=1, a_kmajor=1, b_kmajor=1, c_fp32=1,
                 nvalid=Ncols)
    print(f"(d) both K-major, 1 slice (persistent long-K kernel) {timed(c1):7.1f} us  {fl / timed(c1) / 1e6:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
