"""LDS bank-conflict table per kernel variant from a tools/gpu_pmc_ablate.sh summary (tools/pmc_summary.py output).

    python tools/pmc_lds_table.py gpurun_out/pmc_ablate_<tag>/summary.txt
"""
import re
import sys


def main():
    txt = open(sys.argv[1]).read()
    for b in re.split(r'\n(?=\S)', txt):
        lines = b.strip().splitlines()
        if not lines or ('grad_kernel' not in lines[0] and 'raster_kernel' not in lines[0]):
            continue
        d = {}
        for ln in lines[1:]:
            p = ln.split()
            if len(p) == 2:
                d[p[0]] = float(p[1])
        m = re.search(r'median dur ([\d.]+)', lines[0])
        ia, bc = d.get('SQ_LDS_IDX_ACTIVE', 0), d.get('SQ_LDS_BANK_CONFLICT', 0)
        print("%-52s dur %6s us  LDS-active %9.0f  conflicts %9.0f (%4.1f %%)  LDS insts %8.0f  VALU %9.0f  "
              "LDS issue waits %9.0f" % (lines[0].split('  median')[0][:52], m.group(1) if m else '?', ia, bc,
                                         100 * bc / ia if ia else 0, d.get('SQ_INSTS_LDS', 0),
                                         d.get('SQ_INSTS_VALU', 0), d.get('SQ_WAIT_INST_LDS', 0)))


if __name__ == "__main__":
    main()
