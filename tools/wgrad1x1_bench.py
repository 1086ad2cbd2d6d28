"""1x1 weight gradients (dW[O][C] = sum_t dY[t][o] X[t][c], both operands token-major) of the
train step: the engine's current choice against split-K fp32 slices + fixed-order sum at
several slice counts.  us per call (GEMM + slice sum), TF/s, rel error vs fp32."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FS2_HIP_LIB", os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd",
                                                  "fastspeech2", "libfs2_hip_exp.so"))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402
from fastspeech2 import ops  # noqa: E402
from fastspeech2.engine import wgrad_slices, eff_split  # noqa: E402


def timed(fn, n=20):
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


SHAPES = [("dec in_proj", 31264, 1152, 384), ("dec out_proj", 31264, 384, 384),
          ("dec conv2", 31264, 384, 1536), ("enc in_proj", 6400, 1152, 384),
          ("enc out_proj", 6400, 384, 384), ("enc conv2", 6400, 384, 1536),
          ("concat_proj", 6400, 384, 776), ("mel linear", 31264, 80, 384)]


def main():
    bf = torch.bfloat16
    only = os.environ.get("WG_ONLY")
    for name, T, O, C in SHAPES:
        if only and only not in name:
            continue
        torch.manual_seed(T + O + C)
        dY = (torch.randn(T, O, device="cuda") * 0.5).to(bf)
        X = (torch.randn(T, C, device="cuda") * 0.5).to(bf)
        ref = dY.float().t() @ X.float()
        K = (T + 7) // 8 * 8
        G = torch.zeros(O, C, device="cuda")
        fl = 2.0 * T * O * C
        ws = torch.empty(64 * O * C, device="cuda")

        def engine():
            ns = eff_split(K, wgrad_slices(O, C, C, K, 1), 64)
            if ns == 1 and O * C > 600_000:
                ns = eff_split(K, max(1, min(-(-240 // (-(-O // 256) * -(-C // 256))), (K // 64) // 8)), 64)
            if ns > 1:
                st = O * C
                ops.gemm(O, C, K, dY, O, X, C, ws, C, dt=1, a_kmajor=0, b_kmajor=0, c_fp32=1,
                         kvalid=T, nvalid=C, split_k=ns, split_stride=st)
                ops.sum_slices(ws, ns, st, st, G, accumulate=1)
                return ns
            tiles = -(-O // 128) * -(-C // 128)
            split = max(1, min(-(-512 // tiles), K // 256)) if tiles < 256 else 1
            ops.gemm(O, C, K, dY, O, X, C, G, C, dt=1, a_kmajor=0, b_kmajor=0, c_fp32=1,
                     kvalid=T, nvalid=C, accumulate=1, split_k=split)
            return -split
        G.zero_()
        how = engine()
        torch.cuda.synchronize()
        err = ((G - ref).abs().max() / ref.abs().max()).item()
        us = timed(engine)
        print(f"{name:13s} O={O:5d} C={C:5d} T={T:6d} engine({how:+d})  {us:7.1f} us "
              f"{fl / us / 1e6:6.0f} TF/s rel {err:.1e}", flush=True)
        for ns in (4, 8, 12, 16, 24, 32, 48):
            nse = eff_split(K, ns, 64)
            st = O * C

            def sl():
                ops.gemm(O, C, K, dY, O, X, C, ws, C, dt=1, a_kmajor=0, b_kmajor=0, c_fp32=1,
                         kvalid=T, nvalid=C, split_k=nse, split_stride=st)
                ops.sum_slices(ws, nse, st, st, G, accumulate=1)
            G.zero_()
            sl()
            torch.cuda.synchronize()
            err = ((G - ref).abs().max() / ref.abs().max()).item()
            us = timed(sl)
            print(f"{name:13s} O={O:5d} C={C:5d} T={T:6d} slices {nse:3d}  {us:7.1f} us "
                  f"{fl / us / 1e6:6.0f} TF/s rel {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
