"""Summarise rocprofv3 --pmc CSV passes (tools/pmc_chain.sh) per kernel.

usage: python tools/pmc_summary.py gpurun_out/pmc [--json out.json] [--md out.md]

Every pass directory holds run_counter_collection.csv (one row per dispatch x
counter).  Values are averaged per dispatch for each kernel.  HBM traffic
follows MI355X_MICROARCH.md "HBM": FETCH_SIZE (KB) reports half the bytes of a
16-B/lane streaming read on gfx950 -> x2; WRITE_SIZE (KB) is exact for
16-B/lane stores.  Derived: VALU/MFMA, LDS bank-conflict fraction, wave stall
split.
"""

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


_DEM = {}


def demangle(name):
    if name.startswith("_Z") and name not in _DEM:
        import subprocess
        try:
            # c++filt predates the DF16b (__bf16) mangling: spell it as a vendor type
            fixed = name.replace("DF16b", "u4bf16")
            _DEM[name] = subprocess.run(["c++filt", fixed], capture_output=True, text=True).stdout.strip()
        except OSError:
            _DEM[name] = name
    return _DEM.get(name, name)


def short(name):
    name = demangle(name)
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name) if "<" not in name else name
    name = re.sub(r"\((ConvParams|ChainParams|.*Params)\)$", "", name)
    name = name.replace("__hip_bfloat16", "bf16").replace("__bf16", "bf16")
    return name.split("(")[0] if name.count("(") and not name.startswith("(") else name


def load(root):
    per = defaultdict(lambda: defaultdict(list))    # kernel -> counter -> [per-dispatch]
    meta = {}
    for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        disp = defaultdict(dict)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                key = (k, row["Dispatch_Id"])
                disp[key][row["Counter_Name"]] = disp[key].get(row["Counter_Name"], 0.0) + \
                    float(row["Counter_Value"])
                meta.setdefault(k, {"vgpr": int(row["VGPR_Count"]), "agpr": int(row["Accum_VGPR_Count"]),
                                    "lds": int(row["LDS_Block_Size"]), "scratch": int(row["Scratch_Size"])})
        for (k, _), cs in disp.items():
            for c, v in cs.items():
                per[k][c].append(v)
    out = {}
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["dispatches"] = max(len(v) for v in cs.values())
        r = dict(meta[k])
        r["mean"] = m
        if "FETCH_SIZE" in m:
            r["hbm_read_bytes"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            r["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in r and "hbm_write_bytes" in r:
            r["hbm_bytes"] = r["hbm_read_bytes"] + r["hbm_write_bytes"]
        if m.get("SQ_INSTS_MFMA"):
            r["valu_per_mfma"] = m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"]
        if m.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
        # MFMA utilisation (MI355X_MICROARCH.md "rocprofv3 PMC"): busy cycles
        # summed over the 1024 SIMDs against the dispatch's cycles, GRBM_GUI_ACTIVE
        # being the sum over the 8 XCDs (per-XCD cycles = GUI / 8)
        if m.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            cyc = m["GRBM_GUI_ACTIVE"] / 8.0
            r["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc)
            r["gui_cycles"] = cyc
            if m.get("SQ_INSTS_MFMA"):
                # 16x16x32 bf16: 16 cycles per MFMA per SIMD (cycle-constants table)
                r["mfma_issue_frac"] = m["SQ_INSTS_MFMA"] * 16.0 / (1024.0 * cyc)
        if m.get("SQ_WAVE_CYCLES"):
            w = m["SQ_WAVE_CYCLES"]
            r["wait_frac"] = m.get("SQ_WAIT_ANY", 0) / w
            r["issue_stall_frac"] = m.get("SQ_WAIT_INST_ANY", 0) / w
            r["active_frac"] = m.get("SQ_ACTIVE_INST_ANY", 0) / w
        out[k] = r
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    ap.add_argument("--md")
    a = ap.parse_args()
    s = load(a.root)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(s, f, indent=1, sort_keys=True)
    rows = ["| kernel | disp | VGPR/AGPR | LDS B | VALU/MFMA | LDS confl | wait / stall / active | HBM read MB | HBM write MB | MFMA busy |",
            "|---|---|---|---|---|---|---|---|---|---|"]
    key = lambda kv: -kv[1].get("hbm_bytes", 0) - kv[1]["mean"].get("SQ_INSTS_MFMA", 0)
    for k, r in sorted(s.items(), key=key):
        if k.startswith("__amd"):
            continue
        f = lambda x, fmt: (fmt % x) if x is not None else "-"
        rows.append("| %s | %d | %d/%d | %d | %s | %s | %s | %s | %s | %s |" % (
            k, r["mean"]["dispatches"], r["vgpr"], r["agpr"], r["lds"],
            f(r.get("valu_per_mfma"), "%.1f"), f(r.get("lds_conflict_frac"), "%.2f"),
            ("%.2f / %.2f / %.2f" % (r["wait_frac"], r["issue_stall_frac"], r["active_frac"]))
            if "wait_frac" in r else "-",
            f(r.get("hbm_read_bytes", None) and r["hbm_read_bytes"] / 1e6, "%.1f"),
            f(r.get("hbm_write_bytes", None) and r["hbm_write_bytes"] / 1e6, "%.1f"),
            f(r.get("mfma_busy_frac"), "%.3f")))
    txt = "\n".join(rows)
    if a.md:
        with open(a.md, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
