"""cProfile the headline sweep loop (host overhead between kernel launches)."""
import os
import cProfile
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/host_profile.txt"
prof = cProfile.Profile()
prof.enable()
bench.main(["--steps", "60", "--warmup", "10"])
prof.disable()
with open(out, "w") as f:
    st = pstats.Stats(prof, stream=f)
    st.sort_stats("cumulative").print_stats(60)
    st.sort_stats("tottime").print_stats(40)
