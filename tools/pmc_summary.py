"""Summarise the per-counter rocprofv3 --pmc passes of `tools/gpu_session.sh pmc`
into profiles/pmc_traffic.json (the `traffic` field of bench.py's roofline).

Usage: python tools/pmc_summary.py GPURUN_OUT_DIR ROUND_TAG
Averages each counter over the k_chunks dispatches of its pass (the config-2
launch shape: 1 M x 32 KiB, LDS-DMA loader) and applies the gfx950 HBM
correction of MI355X_MICROARCH.md: bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024.
Copies the raw counter CSVs to profiles/<ROUND_TAG>/pmc_<counter>.csv.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BS, NBLK = 32768, 1 << 20


def main():
    src, tag = sys.argv[1], sys.argv[2]
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    vals = {}
    for d in sorted(glob.glob(os.path.join(src, "pmc_*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.isfile(f):
            continue
        name = os.path.basename(d)[4:]
        shutil.copy(f, os.path.join(dst, "pmc_%s.csv" % name))
        per = {}
        for row in csv.DictReader(open(f)):
            if "k_chunks" not in row["Kernel_Name"]:
                continue
            key = row["Dispatch_Id"]
            per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        if per:
            vals[name] = sum(per.values()) / len(per)
    out = {}
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.isfile(path):
        out = json.load(open(path))
    ncomp = NBLK * (BS // 128)
    ent = {
        "hbm_bytes_per_launch": int(vals["FETCH_SIZE"] * 1024 * 2 + vals["WRITE_SIZE"] * 1024),
        "algorithmic_bytes_per_launch": NBLK * (BS + 32),
        "FETCH_SIZE_kb": vals["FETCH_SIZE"],
        "WRITE_SIZE_kb": vals["WRITE_SIZE"],
        "correction": "hbm = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (gfx950: FETCH_SIZE reads half of "
                      "a wide coalesced stream, MI355X_MICROARCH.md HBM)",
    }
    for k in ("SQ_INSTS_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY",
              "SQ_ACTIVE_INST_VALU"):
        if k in vals:
            ent[k] = vals[k]
    if "SQ_INSTS_VALU" in vals:
        # SQ_INSTS_VALU counts wave instructions: x64 lanes / compressions
        ent["valu_lane_instr_per_compression"] = vals["SQ_INSTS_VALU"] * 64 / ncomp
    ent["source"] = ("profiles/%s/pmc_*.csv (rocprofv3 --pmc, one counter per pass, "
                     "bench.py --steps 3 --warmup 1)" % tag)
    out["bs32768/n1048576/glds"] = ent
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")
    print(json.dumps(ent, indent=1))


if __name__ == "__main__":
    main()
