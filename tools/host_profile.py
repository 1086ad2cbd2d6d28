"""cProfile of the host side of the bench step (B=32 bf16 eager), steps only (model build and
warm-up outside the profile): where the Python / ctypes enqueue time per step goes.  Prints the
top functions by self time and by cumulative time, and the uninstrumented host time per step."""
import cProfile
import os
import pstats
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def main():
    from fastspeech2 import load_config
    from fastspeech2.model import FastSpeech2
    from fastspeech2.train import FusedTrainer
    from fastspeech2.synthetic import make_batch, as_tuple
    cfg = load_config()
    torch.manual_seed(0)
    model = FastSpeech2(**cfg["model"]["fastspeech2"], n_speakers=4,
                        act_dtype=torch.bfloat16).cuda().train()
    tr = FusedTrainer(model, lr=cfg["train"]["learning_rate"])
    tr.use_graph = False
    b = make_batch(B=32, seed=0, device="cuda")
    bt, inten = as_tuple(b)
    Tm = b["mel"].shape[1]
    for _ in range(3):
        tr.step(bt, inten, mel_len_max=Tm)
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        tr.step(bt, inten, mel_len_max=Tm)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"uninstrumented: host {(t1 - t0) / n * 1e3:.2f} ms/step, wall {(t2 - t0) / n * 1e3:.2f} "
          f"ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        tr.step(bt, inten, mel_len_max=Tm)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr, stream=sys.stdout)
    st.sort_stats("tottime").print_stats(40)
    st.sort_stats("cumtime").print_stats(40)


if __name__ == "__main__":
    main()
