"""Per-(kernel, grid) summary of a rocprofv3 --kernel-trace CSV: calls,
median / mean / min / max duration (µs) for every kernel AND grid size, so a
bench line's roofline fraction can be recomputed from profiles/ alone (the
plain --stats summary averages every grid of a kernel together: C3's
8,192-stripe and c3s8's 1,024-stripe launches of k_encode_ws).

    python tools/grid_stats.py gpurun_out/prof_default/run_kernel_trace.csv > profiles/r04/x_kernel_grid_stats.csv
"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    rows = defaultdict(list)
    for path in sys.argv[1:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                grid = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
                wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                rows[(r["Kernel_Name"], grid, wg)].append(dur)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid_threads", "workgroup", "workgroups", "calls", "median_us", "mean_us", "min_us",
                "max_us", "total_us"])
    for (name, grid, wg), d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        threads = grid[0] * grid[1] * grid[2]
        w.writerow([name, "x".join(map(str, grid)), wg, threads // max(1, wg), len(d),
                    round(statistics.median(d), 2), round(statistics.fmean(d), 2), round(min(d), 2),
                    round(max(d), 2), round(sum(d), 1)])


if __name__ == "__main__":
    main()
