"""Summary of tools/calib_valu.sh: what gfx950's SQ counters read for kernels
of known behaviour, and k_raster's wave-cycle split per ablation phase.

Calibration (tools/calib_valu.hip): for each kernel, the counters against the
instructions it is known to issue and the cycles it ran
(GRBM_GUI_ACTIVE / 8 XCDs = cycles per XCD; MI355X_MICROARCH.md "DVFS").
The VALU pipe of a SIMD-32 takes 2 cycles per wave64 instruction
(MI355X_MICROARCH.md:54, :473), so k_fma_indep<W>'s known pipe occupancy is
insts_per_SIMD x 2 / cycles; `valu_pipe_factor` is the factor f for which
SQ_ACTIVE_INST_VALU x f / (1,024 SIMDs x cycles) equals that occupancy.

Usage: python3 tools/calib_valu_summary.py gpurun_out/r06/calib
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

N_CU, N_SIMD, N_XCD = 256, 1024, 8


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("csg::", "").replace("void ", "")
    n = n.split("(")[0].strip()
    return re.sub(r"\s+", "", n)


def load_pass(d, pick="last"):
    """{kernel: {counter: value}} of one pass directory.  pick='last': the
    kernel's last dispatch (calibration: skips the warm-up); 'grid': the mean
    over the dispatches with the kernel's largest grid (bench: skips the
    sizing pass's small chains)."""
    rows = defaultdict(lambda: defaultdict(dict))   # kernel -> dispatch -> counter -> value
    grid, dur = {}, defaultdict(dict)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = short(r.get("Kernel_Name", ""))
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            rows[k][did][r["Counter_Name"]] = rows[k][did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            g = int(r.get("Grid_Size") or 0)
            grid[(k, did)] = g
            try:
                dur[k][did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
            except (KeyError, ValueError):
                pass
    out = {}
    for k, ds in rows.items():
        if pick == "last":
            sel = [max(ds)]
        else:
            gmax = max(grid[(k, x)] for x in ds)
            sel = [x for x in ds if grid[(k, x)] == gmax]
        agg = defaultdict(float)
        for x in sel:
            for c, v in ds[x].items():
                agg[c] += v / len(sel)
        ms = [dur[k][x] for x in sel if x in dur[k]]
        if ms:
            agg["dispatch_ms"] = sum(ms) / len(ms)
        agg["dispatches"] = len(sel)
        out[k] = dict(agg)
    return out


def merge(dirs, pick):
    m = defaultdict(dict)
    for d in dirs:
        for k, c in load_pass(d, pick).items():
            for n, v in c.items():
                if n in ("dispatch_ms", "dispatches") and n in m[k]:
                    continue
                m[k][n] = v
    return m


def split(c):
    """Wave-cycle split and pipe occupancy of one kernel's counters."""
    o = {}
    wc = c.get("SQ_WAVE_CYCLES")
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / N_XCD
    if wc:
        for n, key in (("SQ_WAIT_ANY", "parked_wait_any"), ("SQ_WAIT_INST_ANY", "issue_stall_wait_inst_any"),
                       ("SQ_ACTIVE_INST_ANY", "issuing_active_inst_any")):
            if n in c:
                o[key] = round(c[n] / wc, 4)
    if cyc > 0:
        o["cycles_per_xcd"] = round(cyc)
        if wc:
            # SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md:488): waves resident per SIMD
            o["waves_per_simd"] = round(wc * 4 / N_SIMD / cyc, 3)
        if "SQ_INSTS_VALU" in c:
            o["valu_pipe_occupancy"] = round(c["SQ_INSTS_VALU"] * 2 / N_SIMD / cyc, 4)
        if "SQ_ACTIVE_INST_VALU" in c:
            o["formula_r05_active_x4"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / N_SIMD / cyc, 4)
            o["active_x2"] = round(c["SQ_ACTIVE_INST_VALU"] * 2 / N_SIMD / cyc, 4)
    if c.get("SQ_INSTS_VALU") and "SQ_ACTIVE_INST_VALU" in c:
        o["active_per_valu_inst"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_INSTS_VALU"], 4)
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        o["lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64), 4)
    for n in c:
        if re.search("BARRIER|SLEEP", n):
            o[n.lower() + "_share"] = round(c[n] / wc, 4) if wc else None
    return o


def main(root):
    res = {"calibration": {}, "raster_phases": {}, "production": {}}
    meta = json.load(open(os.path.join(root, "calib.json")))
    known = {k["name"].replace(" ", ""): k for k in meta["kernels"]}
    cal = merge([d for d in sorted(glob.glob(os.path.join(root, "calib_*"))) if os.path.isdir(d)], "last")
    for name, c in cal.items():
        kn = known.get(name)
        if kn is None:
            continue
        e = {"ms_hip_event": kn["ms"], "waves": kn["waves"], **{k: round(v, 1) for k, v in c.items()}}
        e.update(split(c))
        if kn["valu_per_wave"]:
            want = kn["valu_per_wave"] * kn["waves"]
            e["valu_insts_expected"] = want
            e["insts_ratio"] = round(c.get("SQ_INSTS_VALU", 0) / want, 4)
        res["calibration"][name] = e
    # the factor that maps SQ_ACTIVE_INST_VALU onto pipe occupancy, from the saturated case
    sat = res["calibration"].get("k_fma_indep<8>")
    if sat and sat.get("SQ_ACTIVE_INST_VALU"):
        cyc = sat["cycles_per_xcd"]
        occ = sat["SQ_INSTS_VALU"] * 2 / N_SIMD / cyc   # known: 2 cycles per wave64 v_fma_f32
        res["valu_pipe_factor"] = round(occ * N_SIMD * cyc / sat["SQ_ACTIVE_INST_VALU"], 4)
        res["saturated_occupancy"] = round(occ, 4)
    for d in sorted(glob.glob(os.path.join(root, "raster_d*_*"))):
        if not os.path.isdir(d):
            continue
        dbg = os.path.basename(d).split("_")[1]
        m = load_pass(d, "grid")
        for k in ("k_raster<false>", "k_raster"):
            if k in m:
                ph = res["raster_phases"].setdefault(dbg, {})
                ph.update({n: round(v, 1) for n, v in m[k].items()})
                ph.update(split(ph))
    prod = merge([d for d in sorted(glob.glob(os.path.join(root, "prod_*"))) if os.path.isdir(d)], "grid")
    for k in ("k_raster<false>", "k_setup", "k_bin<false>", "k_count<false>"):
        if k in prod:
            e = {n: round(v, 1) for n, v in prod[k].items()}
            e.update(split(prod[k]))
            res["production"][k] = e
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
