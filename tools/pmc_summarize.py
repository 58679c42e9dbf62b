"""Summarise rocprofv3 --pmc CSV passes per kernel (average per dispatch).

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: bytes =
FETCH_SIZE*1024*2 (gfx950 FETCH_SIZE counts half the bytes of a wide read)
+ WRITE_SIZE*1024.  Prints JSON; with --write-profile also updates
profiles/pmc_traffic.json for bench.py's roofline.traffic field.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N_CU = 256
N_SIMD = N_CU * 4   # MI355X: 256 CUs x 4 SIMDs
N_XCD = 8
# VALU pipe occupancy that 8 waves per SIMD of independent v_fma_f32 reach on the MI355X
# (k_fma_indep<8>, profiles/r06/calib/summary.json): the practical ceiling for a kernel
VALU_PIPE_CEILING = 0.80


def _grid(row):
    if "Grid_Size" in row:
        return int(row["Grid_Size"] or 0)
    g = 1
    for a in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"):
        g *= int(row.get(a) or 1)
    return g


def load(d):
    """Per kernel and counter, the values of the dispatches with the kernel's
    largest grid: bench.py's sizing pass (csg_size_work) launches the setup
    and binning kernels on 64-frame chains before the timed steps, and those
    dispatches are not the bench's launches."""
    rows = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            name = row.get("Kernel_Name", "")
            short = (name.replace("(anonymous namespace)::", "").split("(")[0].replace("csg::", "")
                     .replace("void ", "").split("<")[0].strip())
            rows[short].append((_grid(row), row["Counter_Name"], float(row["Counter_Value"])))
    per = defaultdict(lambda: defaultdict(list))
    for short, rs in rows.items():
        gmax = max(g for g, _, _ in rs)
        for g, c, v in rs:
            if g == gmax:
                per[short][c].append(v)
    return per


def main(root, write_profile=False, workload="C3", frames_per_launch=60):
    out = {}
    for sub in sorted(os.listdir(root)):
        p = os.path.join(root, sub)
        if not os.path.isdir(p):
            continue
        for k, ctrs in load(p).items():
            o = out.setdefault(k, {})
            for c, vals in ctrs.items():
                o[c] = sum(vals) / len(vals)
                o[c + "_n"] = len(vals)
    for k, o in out.items():
        if "FETCH_SIZE" in o and "WRITE_SIZE" in o:
            o["hbm_bytes_per_launch"] = o["FETCH_SIZE"] * 1024 * 2 + o["WRITE_SIZE"] * 1024
        if "GRBM_GUI_ACTIVE" in o and o["GRBM_GUI_ACTIVE"] > 0:
            cyc = o["GRBM_GUI_ACTIVE"] / N_XCD   # GRBM_GUI_ACTIVE is summed over the 8 XCDs
            # VALU pipe occupancy, calibrated on gfx950 (tools/calib_valu.hip, profiles/r06/calib):
            # SQ_ACTIVE_INST_VALU counts ONE per wave64 VALU instruction (= SQ_INSTS_VALU, at 1 and
            # at 8 waves per SIMD alike), and a SIMD-32 pipe takes 2 cycles per wave64 instruction
            # (MI355X_MICROARCH.md:54, :473); 8 waves per SIMD of independent v_fma_f32 reach 0.80.
            # (Round 5's formula, SQ_ACTIVE_INST_VALU x 4 / SIMDs / cycles, is twice this and
            # exceeded 1.)
            n_valu = o.get("SQ_INSTS_VALU", o.get("SQ_ACTIVE_INST_VALU"))
            if n_valu is not None:
                o["valu_pipe_occupancy"] = n_valu * 2 / N_SIMD / cyc
            if "SQ_THREAD_CYCLES_VALU" in o and o.get("SQ_ACTIVE_INST_VALU", 0) > 0:
                o["valu_lane_util"] = o["SQ_THREAD_CYCLES_VALU"] / (o["SQ_ACTIVE_INST_VALU"] * 64)
            if o.get("SQ_WAVE_CYCLES"):
                # wave-cycles: parked on s_waitcnt / s_barrier (SQ_WAIT_ANY), stalled with an
                # instruction ready (SQ_WAIT_INST_ANY), issuing (SQ_ACTIVE_INST_ANY); disjoint
                wc = o["SQ_WAVE_CYCLES"]
                o["wave_cycles"] = {k: round(o[c] / wc, 4) for k, c in (("parked", "SQ_WAIT_ANY"),
                                    ("issue_stall", "SQ_WAIT_INST_ANY"), ("issuing", "SQ_ACTIVE_INST_ANY")) if c in o}
                o["waves_per_simd"] = wc * 4 / N_SIMD / cyc   # SQ_WAVE_CYCLES in quad-cycles
        if "SQ_LDS_IDX_ACTIVE" in o and o["SQ_LDS_IDX_ACTIVE"] > 0:
            # LDS-array cycles (summed over the 256 CUs) and the extra cycles bank conflicts
            # added to them (MI355X_MICROARCH.md §LDS): conflict share and LDS busy per CU
            if "SQ_LDS_BANK_CONFLICT" in o:
                o["lds_conflict_share"] = o["SQ_LDS_BANK_CONFLICT"] / o["SQ_LDS_IDX_ACTIVE"]
            if "GRBM_GUI_ACTIVE" in o and o["GRBM_GUI_ACTIVE"] > 0:
                o["lds_busy"] = o["SQ_LDS_IDX_ACTIVE"] / N_CU / (o["GRBM_GUI_ACTIVE"] / N_XCD)
        if "SQ_WAIT_INST_LDS" in o and o.get("SQ_WAVE_CYCLES"):
            o["lds_wait_share"] = o["SQ_WAIT_INST_LDS"] / o["SQ_WAVE_CYCLES"]
    print(json.dumps(out, indent=1, sort_keys=True))
    if write_profile and "k_raster" in out and "hbm_bytes_per_launch" in out["k_raster"]:
        # the bench line of a pass names the workload, frames per launch and B_frame it ran
        line = None
        for f in sorted(glob.glob(os.path.join(root, "*.json"))):
            try:
                line = json.load(open(f))
                break
            except Exception:
                continue
        here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        prof = {"workload": line["config"]["workload"].split(":")[0] if line else workload,
                "frames_per_launch": line["config"]["frames_per_launch"] if line else frames_per_launch,
                "B_frame": (line["roofline"].get("B_frame") or line["roofline"].get("frame_level", {}).get("B_frame"))
                if line else None,
                "bytes_per_launch": {k: int(out[k]["hbm_bytes_per_launch"]) for k in ("k_raster", "k_setup")
                                     if "hbm_bytes_per_launch" in out.get(k, {})},
                "k_raster_fetch_size_kb": out["k_raster"]["FETCH_SIZE"],
                "k_raster_write_size_kb": out["k_raster"]["WRITE_SIZE"],
                "correction": "FETCH_SIZE x2 (gfx950 counts 64 B per 128-B read request: TCC_EA0_RDREQ x 64 B; "
                              "MI355X_MICROARCH.md §HBM), WRITE_SIZE x1; KB = 1024 B. Basis for k_raster's access "
                              "mix: profiles/r01/fetch_calibration.json (4-B gathers and 112-B records also cost "
                              "one 128-B request per touched line)",
                "k_raster_valu_pipe_occupancy": out["k_raster"].get("valu_pipe_occupancy"),
                "valu_pipe_ceiling": VALU_PIPE_CEILING,
                "k_raster_wave_cycles": out["k_raster"].get("wave_cycles"),
                "k_raster_valu_lane_util": out["k_raster"].get("valu_lane_util"),
                "source": os.path.basename(os.path.normpath(root))}
        path = os.path.join(here, "profiles", "pmc_traffic.json")
        try:   # per-frame work counts (profiling counters) do not depend on the launch size: keep them
            keep = json.load(open(path)).get("k_raster_work_per_frame")
            if keep:
                prof["k_raster_work_per_frame"] = keep
        except Exception:
            pass
        json.dump(prof, open(path, "w"), indent=1)


if __name__ == "__main__":
    fpl = 240
    for a in sys.argv[2:]:
        if a.startswith("--frames-per-launch="):
            fpl = int(a.split("=", 1)[1])
    main(sys.argv[1], "--write-profile" in sys.argv, frames_per_launch=fpl)
