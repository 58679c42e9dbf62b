#!/bin/bash
# FETCH_SIZE calibration (see calib_fetch.hip): one PMC pass, one kernel-trace pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/calib
mkdir -p $OUT
[ -x tools/calib_fetch ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/calib_fetch.hip -o tools/calib_fetch || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- ./tools/calib_fetch > $OUT/calib.json &&
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/req -o pmc -- ./tools/calib_fetch > /dev/null
rc=$?
python3 - <<'PY'
import csv, glob, json, collections
out = json.load(open("gpurun_out/calib/calib.json"))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in ("fetch", "req"):
    for p in glob.glob(f"gpurun_out/calib/{d}/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
ref = {"k_gather4": out["gather4_lines_bytes"] + out["index_bytes"], "k_rec112": out["rec112_bytes"] + out["index_bytes"],
       "k_stream16": out["stream16_bytes"]}
res = {}
for k, want in ref.items():
    c = {n: sum(v) / len(v) for n, v in agg[k].items()}
    fs = c.get("FETCH_SIZE", 0) * 1024
    res[k] = {"touched_bytes": want, "FETCH_SIZE_bytes": fs, "ratio": round(fs / want, 3), **{n: v for n, v in c.items() if n != "FETCH_SIZE"}}
print(json.dumps(res, indent=1))
json.dump(res, open("gpurun_out/calib/summary.json", "w"), indent=1)
PY
exit $rc
