"""Per-dispatch PMC means of the frame-path kernels from tools/frame_pmc.sh's rocprofv3 passes.

  python3 tools/frame_pmc.py gpurun_out/framepmc [--out profiles/r02_frame_pmc.json]

Derived figures (MI355X_MICROARCH.md §rocprofv3 PMC slots): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_*
count quad-cycles, so their ratios are fractions of a wave's lifetime; HBM read bytes = FETCH_SIZE
(KiB) x 1024 x 2 (the gfx950 FETCH_SIZE correction bench.py also applies), write = WRITE_SIZE x 1024.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

# every kernel of the frame path: stage A (featureExtraction + VoxelGrid) and stage B (odometry)
STAGE_B = ["k_grid_bounds", "k_grid_count", "k_grid_scan", "k_grid_scatter", "k_assoc", "k_observe", "k_lm_solve",
           "k_rgm_bucket", "k_rgm_finish", "k_rg_append_keys", "k_rg_tail", "k_rg_write", "k_rg_dep"]
# the tie-order sort's kernels run in both stages (VoxelGrid in A, rgbds in B): their means mix the two
BOTH = ["k_tie_medium", "k_tie_mid", "k_tie_local", "k_tie_heap", "k_tie_compact", "k_tie_setup", "k_tie_scan",
        "k_tie_split"]


def short(name):
    """names read "void pf::(anonymous namespace)::k_x<2>(pf::Args)": the k_ identifier"""
    m = re.search(r"\b(k_\w+?)(<|\(|$)", name)
    return m.group(1) if m else ""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default=None)
    ap.add_argument("--source", default="rocprofv3 --pmc passes (tools/frame_pmc.sh) over bench.py --steps 100 "
                                        "--no-graph (configs[1], S64)")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(a.root + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", ""))
            if k:
                # one row per (dispatch, counter): sum over the per-XCD / per-SE dimension rows of a dispatch
                acc[k][(row["Counter_Name"], row.get("Dispatch_Id", ""))].append(float(row["Counter_Value"]))
    out = {"source": a.source, "kernels": {}}
    for k in sorted(acc, key=lambda x: (x not in STAGE_B, x)):
        per = defaultdict(list)
        for (ctr, _), vals in acc[k].items():
            per[ctr].append(sum(vals))
        m = {c: sum(v) / len(v) for c, v in per.items()}
        d = {"stage": "B" if k in STAGE_B else ("A+B" if k in BOTH else "A"), "dispatches": max(len(v) for v in per.values()),
             "mean_per_dispatch": m}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc and m.get("SQ_WAVES"):
            d["wave_cycles_per_wave"] = 4 * wc / m["SQ_WAVES"]          # quad-cycles -> cycles
        if m.get("SQ_BUSY_CYCLES") and m.get("GRBM_GUI_ACTIVE"):
            d["sq_busy_frac_of_gpu_active"] = m["SQ_BUSY_CYCLES"] / m["GRBM_GUI_ACTIVE"]
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in m:
                    d["frac_of_wave_cycles_" + c[3:].lower()] = m[c] / wc
        if m.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if c in m:
                    d[c[3:].lower() + "_per_wave"] = m[c] / m["SQ_WAVES"]
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in m:
            d["hbm_read_bytes"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            d["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        out["kernels"][k] = d
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        open(a.out, "w").write(s + "\n")
    else:
        open(os.path.join(a.root, "frame_pmc.json"), "w").write(s + "\n")


if __name__ == "__main__":
    main()
