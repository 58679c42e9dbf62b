"""Per-kernel dispatch statistics from a rocprofv3 kernel_trace.csv, split by
grid size.  bench.py's sizing pass (csg_size_work) launches k_clip, k_setup,
k_count, k_colscan and k_scan on chains of 64 frames before the timed steps;
rocprofv3's --stats summary averages them with the bench's own launches.  This
separates them: one row per (kernel, grid), calls / average / min / max ms.

    python tools/kernel_stats_by_grid.py gpurun_out/prof_r04/kt_kernel_trace.csv [--top 12]
"""
import csv
import sys
from collections import defaultdict


def main(path, top=12):
    rows = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        grid = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        rows[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = sorted(rows.items(), key=lambda kv: -sum(kv[1]))[:top]
    print(f"{'kernel':42s} {'grid':>22s} {'calls':>6s} {'avg_ms':>10s} {'min_ms':>10s} {'max_ms':>10s} {'total_ms':>10s}")
    for (name, grid), ts in out:
        print(f"{name[:42]:42s} {str(grid):>22s} {len(ts):6d} {sum(ts) / len(ts):10.4f} {min(ts):10.4f} "
              f"{max(ts):10.4f} {sum(ts):10.2f}")


if __name__ == "__main__":
    top = 12
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
    main(sys.argv[1], top)
