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


def batch_rows(f):
    """Rows of a config-3 PMC csv that belong to the bench's batches: those
    after the splitmix64 fill (cir_init's warm-up hashes come before it),
    without the fill and the runtime's copy/fill kernels."""
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    fill = min(int(r["Dispatch_Id"]) for r in rows if "k_fill_splitmix64" in r["Kernel_Name"])
    return [r for r in rows if int(r["Dispatch_Id"]) > fill and "__amd_rocclr" not in r["Kernel_Name"]]


def config3(src, tag):
    """`pmc3t` passes: FETCH_SIZE / WRITE_SIZE summed over every kernel of a
    config-3 batch (ordering, quad part, lane part, relay checks), per batch
    (= per k_chain_keys dispatch), into pmc_traffic.json["config3"].  The
    `pmcreq` pass (TCC_EA0_RDREQ / _32B / TCC_BUBBLE) shows the request size
    behind FETCH_SIZE's factor 2 for this access pattern too."""
    sys.path.insert(0, ROOT)
    import bench
    offs, lens, _ = bench.config3_layout()
    algo = int(lens.astype("int64").sum()) + 32 * int(lens.size)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)

    def tally(f):
        per, batches = {}, set()
        for row in batch_rows(f):
            name = row["Kernel_Name"]
            if "k_chain_keys" in name:
                batches.add(row["Dispatch_Id"])
            short = name.split("(")[0].split("::")[-1]
            key = (row["Counter_Name"], short)
            per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        nb = max(1, len(batches))
        return {k: v / nb for k, v in per.items()}, nb

    per_kernel, vals = {}, {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(src, "pmc3t_" + c, "run_counter_collection.csv")
        shutil.copy(f, os.path.join(dst, "pmc3t_%s.csv" % c))
        per, nb = tally(f)
        per_kernel[c] = {k: round(v, 1) for (_, k), v in per.items()}
        vals[c] = sum(per.values())
    ent = {
        "hbm_bytes_per_batch": int(vals["FETCH_SIZE"] * 1024 * 2 + vals["WRITE_SIZE"] * 1024),
        "algorithmic_bytes_per_batch": algo,
        "batches": nb,
        "FETCH_SIZE_kb": round(vals["FETCH_SIZE"], 1), "WRITE_SIZE_kb": round(vals["WRITE_SIZE"], 1),
        "per_kernel_kb": per_kernel,
        "correction": "hbm = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM)",
    }
    ent["ratio_to_algorithmic"] = round(ent["hbm_bytes_per_batch"] / algo, 4)
    req = os.path.join(src, "pmcreq_c3", "run_counter_collection.csv")
    if os.path.isfile(req):
        shutil.copy(req, os.path.join(dst, "pmcreq_c3.csv"))
        per, _ = tally(req)
        tot = {}
        for (c, _), v in per.items():
            tot[c] = tot.get(c, 0.0) + v
        ent["read_requests_per_batch"] = {k: int(v) for k, v in sorted(tot.items())}
        ent["read_bytes_at_128B_per_request"] = int(tot.get("TCC_EA0_RDREQ_sum", 0) * 128)
        ent["request_note"] = ("TCC_BUBBLE (128-B requests) and TCC_EA0_RDREQ_32B read ~0, so "
                               "FETCH_SIZE tallies every request at 64 B; TCC_EA0_RDREQ x 128 B "
                               "matches the bytes read, as for config 2's k_chunks "
                               "(pmcreq_c2.csv): the factor 2 holds for this pattern")
    ent["source"] = ("profiles/%s/pmc3t_*.csv, pmcreq_c3.csv (rocprofv3 --pmc, one pass per "
                     "counter set, bench.py --workload config3 --steps 2 --warmup 1; the "
                     "dispatches of cir_init's warm-up and the data fill excluded)" % tag)
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    out = json.load(open(path)) if os.path.isfile(path) else {}
    out["config3"] = ent
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")
    print(json.dumps(ent, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[3] == "config3":
        config3(sys.argv[1], sys.argv[2])
    else:
        main()
