"""Resource usage and instruction mix of one kernel in a `make asm` listing.

usage: python tools/asm_stats.py build/asm/<name>.s <mangled-name-prefix> [ds|all]
"""
import collections
import re
import sys


def main():
    path, prefix = sys.argv[1], sys.argv[2]
    mode = sys.argv[3] if len(sys.argv) > 3 else "ds"
    txt = open(path).read()
    lines = txt.split("\n")
    s = next(i for i, l in enumerate(lines) if l.startswith(prefix) and ":" in l)
    e = s
    while not lines[e].startswith(".Lfunc_end"):
        e += 1
    c = collections.Counter()
    for l in lines[s:e]:
        m = re.match(r"\s+([a-z_0-9]+)", l)
        if m:
            c[m.group(1)] += 1
    name = lines[s].split(":")[0]
    # the kernel's metadata entry: its fields are listed alphabetically, so the ones before `.name` start at
    # the entry's `- ` line and the ones after it run to the next entry
    at = txt.find(".name:           " + name + "\n")
    start = txt.rfind("\n  - ", 0, at)
    end = txt.find("\n  - ", at)
    meta = txt[start:end if end > 0 else at + 4000]
    for k in (".sgpr_count:", ".vgpr_count:", ".agpr_count:", ".vgpr_spill_count:", ".group_segment_fixed_size:"):
        j = meta.find(k)
        print(meta[j:].split("\n")[0].strip() if j >= 0 else k + " ?")
    print("instructions", sum(c.values()), "ds", sum(v for k, v in c.items() if k.startswith("ds_")),
          "valu", sum(v for k, v in c.items() if k.startswith("v_")))
    for k, v in sorted(c.items(), key=lambda x: -x[1]):
        if mode == "all" or k.startswith("ds_"):
            print("  %-28s %d" % (k, v))


if __name__ == "__main__":
    main()
