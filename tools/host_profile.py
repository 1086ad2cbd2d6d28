"""cProfile of the host side of the bench step (B=32 bf16 eager): where the ~12 ms of Python /
ctypes enqueue time per step goes.  Prints the top functions by total (self) time."""
import cProfile
import os
import pstats
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0], "--steps", "10", "--warmup", "3", "--no-cpu-baseline", "--no-extractor",
            "--no-fp32-leg", "--no-config2-leg"]
import bench  # noqa: E402

pr = cProfile.Profile()
pr.enable()
bench.main()
pr.disable()
st = pstats.Stats(pr, stream=sys.stderr)
st.sort_stats("tottime").print_stats(35)
