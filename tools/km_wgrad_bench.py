"""Conv weight gradient: MN-major implicit conv (conv_mode 3, gemm256_kernel) vs both operands
K-major over padded channel-major images (fs2_pad_transpose + conv_mode 6, gemm_ps_kernel), at
the decoder / encoder FFN conv1 and the PostNet shapes (B=32, bf16).  Prints us per call (GEMM
+ slice sum; the two transposes timed apart) and TF/s of the GEMM's algorithmic FLOPs."""
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


def case(name, B, T, C, O, KW, splits):
    from fastspeech2 import ops
    P = (KW - 1) // 2
    M = B * T
    bf = torch.bfloat16
    dY = (torch.randn(M, O, device="cuda") * 0.5).to(bf)
    X = (torch.randn(M, C, device="cuda") * 0.5).to(bf)
    Ncols = KW * C
    fl = 2.0 * M * O * Ncols
    stride = O * Ncols
    ws = torch.empty(8 * stride, device="cuda")
    out = torch.zeros(O, Ncols, device="cuda")
    K = (M + 7) // 8 * 8
    ns = 3

    def a():
        ops.gemm(O, Ncols, K, dY, O, X, C, ws, Ncols, dt=1, a_kmajor=0, b_kmajor=0,
                 conv=(3, T, KW, C), c_fp32=1, kvalid=M, nvalid=Ncols, split_k=ns,
                 split_stride=stride)
        ops.sum_slices(ws, ns, stride, stride, out, accumulate=1)
    ta = timed(a)
    print(f"{name}: conv3 MN-major (3 slices)     {ta:7.1f} us  {fl / ta / 1e6:6.0f} TF/s", flush=True)
    for S in splits:
        Kp = ops.round_up(B * (T + 2 * P), 64 * S)
        gy = torch.zeros(O * Kp + 128, device="cuda", dtype=bf)
        gx = torch.zeros(C * Kp + 128, device="cuda", dtype=bf)
        dYT, XT = gy[64:64 + O * Kp], gx[64:64 + C * Kp]

        def tr():
            ops.pad_transpose(dY, O, B, T, O, P, 0, dYT, Kp, Kp, dt=1)
            ops.pad_transpose(X, C, B, T, C, P, 1, XT, Kp, Kp, dt=1)
        tt = timed(tr)

        def k():
            ops.gemm(O, Ncols, Kp, dYT, Kp, XT, Kp, ws, Ncols, dt=1, conv=(6, T, KW, C), c_fp32=1,
                     split_k=S, split_stride=stride if S > 1 else 0)
            ops.sum_slices(ws, S, stride, stride, out, accumulate=1)
        tk = timed(k)
        mb = (M * O + M * C) * 2 * 2 / 1e6
        print(f"{name}: conv6 K-major S={S} Kp={Kp}  {tk:7.1f} us  {fl / tk / 1e6:6.0f} TF/s"
              f"  + transposes {tt:6.1f} us ({mb / tt * 1e-3:.2f} TB/s)  total {tk + tt:7.1f}",
              flush=True)
    if os.environ.get("KM_BLAS"):
        # hipBLASLt ceilings (torch.matmul, fp32 out): the plain NT GEMM of the same size with
        # the shifted X rows materialised ([KW*C][Kp]), and the per-tap form (KW GEMMs of
        # O x C x Kp on X's image shifted by j - P elements)
        Kp = ops.round_up(B * (T + 2 * P), 64)
        A = (torch.randn(O, Kp, device="cuda") * 0.5).to(bf)
        Bf = (torch.randn(Ncols, Kp, device="cuda") * 0.5).to(bf)
        tb = timed(lambda: torch.matmul(A, Bf.t()))
        print(f"{name}: hipBLASLt plain {O}x{Ncols}x{Kp}  {tb:7.1f} us  {fl / tb / 1e6:6.0f} TF/s",
              flush=True)
        g = torch.zeros(C * Kp + 128, device="cuda", dtype=bf)
        outp = torch.empty(O, KW, C, device="cuda")

        def taps():
            for j in range(KW):
                xs = g.as_strided((C, Kp), (Kp, 1), 64 + j - P)
                torch.matmul(A, xs.t(), out=outp[:, j, :])
        try:
            tj = timed(taps)
            print(f"{name}: hipBLASLt {KW} tap GEMMs {O}x{C}x{Kp}  {tj:7.1f} us  {fl / tj / 1e6:6.0f} TF/s",
                  flush=True)
        except RuntimeError as e:
            print(f"{name}: per-tap torch.matmul refused: {e}", flush=True)


def main():
    from fastspeech2 import _native
    _native.load()
    case("decoder conv1", 32, 977, 384, 1536, 9, (2, 3, 4))
    case("encoder conv1", 32, 200, 384, 1536, 9, (2, 3))
    if os.environ.get("KM_BLAS"):
        return
    case("postnet mid  ", 32, 977, 512, 512, 5, (6, 12))
    case("postnet pre  ", 32, 977, 80, 512, 5, (6, 12))
    case("postnet post ", 32, 977, 512, 80, 5, (12, 25))
    case("predictor    ", 32, 200, 384, 384, 3, (4, 6))


if __name__ == "__main__":
    main()
