# C2 end-to-end probe (round 6 diagnostics): bench.py end_to_end_line three times on one box
import sys, os
sys.path.insert(0, os.getcwd())
sys.argv = ['bench.py']
import bench
for i in range(3):
    r = bench.end_to_end_line(0, "c2", 400, warm=(i == 0))
    print("C2 e2e", round(r["ms_per_md_step"] * 1e3, 2), "us/MD step", "wall", round(r["wall_s"], 5), flush=True)
