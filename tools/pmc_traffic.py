"""HBM traffic per kernel launch from a tools/gpu_traffic.sh run.

traffic = 2 x FETCH_SIZE + WRITE_SIZE (rocprofv3 reports KB).  The factor 2 is the gfx950 FETCH_SIZE
correction (MI355X_MICROARCH.md, HBM section), confirmed here by the calibration pass: 256 MiB read
once with 4-, 12- and 16-byte lane accesses reports exactly half.  Writes `profiles/<round>/traffic.json`
which bench.py reports as roofline.traffic.

    python tools/pmc_traffic.py gpurun_out/traffic_a profiles/r01/traffic.json
"""
import collections
import csv
import json
import statistics
import sys


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    meta = {}
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter:
            continue
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        vals[k].append(float(r['Counter_Value']))
        meta[k] = {"vgpr": int(r['VGPR_Count']), "sgpr": int(r['SGPR_Count']), "lds": int(r['LDS_Block_Size']),
                   "grid": int(r['Grid_Size']), "wg": int(r['Workgroup_Size'])}
    return {k: statistics.median(v) for k, v in vals.items()}, meta


def main():
    # python tools/pmc_traffic.py SRC DST [TREE]: TREE (the git commit the measured build came from) and the box
    # this runs on are recorded as `measured_on` (run it on the GPU box, after the passes)
    src, dst = sys.argv[1], sys.argv[2]
    tree = sys.argv[3] if len(sys.argv) > 3 else None
    cal, _ = per_kernel(src + '/cal/run_counter_collection.csv', 'FETCH_SIZE')
    fetch, meta = per_kernel(src + '/FETCH_SIZE/run_counter_collection.csv', 'FETCH_SIZE')
    write, _ = per_kernel(src + '/WRITE_SIZE/run_counter_collection.csv', 'WRITE_SIZE')
    cal_bytes = 256 << 20
    factors = {k: cal_bytes / (v * 1024) for k, v in cal.items() if 'read_bytes' in k}
    out = {"method": "2 x FETCH_SIZE + WRITE_SIZE per launch (rocprofv3 --pmc, separate passes, bench.py c3 "
                     "eager launches, median over launches)",
           "fetch_calibration": {k: round(f, 4) for k, f in factors.items()}, "kernels": {}}
    import platform
    box = {"host": platform.node()}
    try:
        import torch
        box["gpu"] = "%s (%s)" % (torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).gcnArchName)
    except Exception:  # noqa: BLE001 -- informative only
        pass
    out["measured_on"] = {"tree": tree, **box}
    for k in sorted(set(fetch) | set(write)):
        if 'fillBuffer' in k or 'read_bytes' in k:
            continue
        fb = 2 * fetch.get(k, 0.0) * 1024
        wb = write.get(k, 0.0) * 1024
        out["kernels"][k] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb),
                             **meta.get(k, {})}
        print("%-24s fetch %8.2f MB  write %8.2f MB  total %8.2f MB  %s" % (k, fb / 1e6, wb / 1e6, (fb + wb) / 1e6,
                                                                        meta.get(k, {})))
    print("calibration factors:", out["fetch_calibration"])
    json.dump(out, open(dst, 'w'), indent=1)


if __name__ == "__main__":
    main()
