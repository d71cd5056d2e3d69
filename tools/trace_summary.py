#!/usr/bin/env python3
"""Per-kernel durations of single-frame launches from a rocprofv3 --kernel-trace CSV (the bench's legs also launch
multi-frame batches, which the --stats average mixes in): count, median and mean of the launches whose grid has one
frame (Grid_Size_Y == 1), for the product instantiations of setup, raster and grad.

    python tools/trace_summary.py gpurun_out/.../run_kernel_trace.csv [bench.json]

With the bench line's JSON, also prints its roofline duration beside the trace's for the roofline kernel."""
import csv
import json
import statistics
import sys

KERNELS = ("setup_kernel<0, 256>", "raster_kernel<3, 0, 0, false, false, false, false, false>",
           "grad_kernel<3, 0, 16, 16, 3>")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    out = {}
    for k in KERNELS:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
             if k in r["Kernel_Name"] and int(r.get("Grid_Size_Y", "1")) == 1]
        if d:
            out[k] = (len(d), statistics.median(d), sum(d) / len(d))
            print("%-60s launches %5d  median %7.2f us  mean %7.2f us" % (k, *out[k]))
    if len(sys.argv) > 2:
        r = json.load(open(sys.argv[2]))["roofline"]
        g = out.get("grad_kernel<3, 0, 16, 16, 3>")
        if g:
            print("bench roofline avg_us %.2f (%s) against the trace's median %.2f: %+.1f %%"
                  % (r["avg_us"], r["avg_us_source"], g[1], 100.0 * (r["avg_us"] / g[1] - 1.0)))


if __name__ == "__main__":
    main()
