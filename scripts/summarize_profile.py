"""Turn a scripts/profile.sh run (gpurun_out/prof, or the directory given after the tag) into
committed evidence under profiles/.

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_kernel_stats.md    per-kernel table with short names
  profiles/pmc_traffic.json         per-kernel HBM bytes per launch from the PMC passes:
                                    FETCH_SIZE x 2 (gfx950 reports half of a wide coalesced
                                    stream, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, KB -> bytes
"""

import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof")
DST = os.path.join(ROOT, "profiles")


def short(name):
    m = re.search(r"(\w+_kernel)(<[^>]*>)?", name)
    return m.group(0) if m else name.split("(")[0][:60]


def main(tag, src=None):
    global SRC
    if src:
        SRC = src
    os.makedirs(DST, exist_ok=True)
    stats = os.path.join(SRC, "trace", "run_kernel_stats.csv")
    if not os.path.exists(stats):  # scripts/gpu_run.sh's prof step writes into the directory itself
        stats = os.path.join(SRC, "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(DST, f"{tag}_kernel_stats.csv"))
        rows = list(csv.DictReader(open(stats)))
        with open(os.path.join(DST, f"{tag}_kernel_stats.md"), "w") as f:
            f.write(f"# rocprofv3 --kernel-trace --stats ({tag})\n\n")
            f.write("| kernel | calls | avg us | total ms | % |\n|---|---|---|---|---|\n")
            for r in rows:
                f.write(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                        f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.2f} |\n")
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        path = os.path.join(SRC, f"pmc_{c}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            pmc[short(r["Kernel_Name"])][c].append(float(r["Counter_Value"]))
    if pmc:
        out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes ({tag})",
               "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch (gfx950)",
               "kernels": {}}
        # one record per kernel base name: the template instance with the most dispatches (the
        # bench's own launch shape; the per-vocab legs run other instances a few times each),
        # every instance listed under "instances"
        for k, d in sorted(pmc.items(), key=lambda kv: -len(kv[1]["FETCH_SIZE"])):
            f = sum(d["FETCH_SIZE"]) / max(1, len(d["FETCH_SIZE"]))
            w = sum(d["WRITE_SIZE"]) / max(1, len(d["WRITE_SIZE"]))
            rec = {"fetch_KB": round(f, 1), "write_KB": round(w, 1), "hbm_bytes_per_launch": int((2 * f + w) * 1024),
                   "dispatches": len(d["FETCH_SIZE"])}
            key = k.split("<")[0]
            if key not in out["kernels"]:
                out["kernels"][key] = dict(rec, instance=k, instances={})
            out["kernels"][key]["instances"][k] = rec
        # kernels the new passes did not profile keep their earlier entries (with their round)
        path = os.path.join(DST, "pmc_traffic.json")
        if os.path.exists(path):
            prev = json.load(open(path))
            for k, v in prev.get("kernels", {}).items():
                if k not in out["kernels"]:
                    out["kernels"][k] = dict(v, round=v.get("round", "earlier"))
        for v in out["kernels"].values():
            v.setdefault("round", tag)
        with open(os.path.join(DST, "pmc_traffic.json"), "w") as fh:
            json.dump(out, fh, indent=1)
    print("profiles written for", tag)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01", sys.argv[2] if len(sys.argv) > 2 else None)
