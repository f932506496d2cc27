#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of `bench.py --pmc-mode`
into HBM bytes per Krylov iteration, following /opt/skills/guides/MI355X_MICROARCH.md
section HBM: counters are in KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of
wide streaming reads, so it is doubled (`--fetch-factor`, default 2) -- our streaming
loads are 8-16 B per lane; see DESIGN.md for the calibration against the pass-2
kernel's exact byte count.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR CONFIG NGPUS K OUT.json
"""
import csv
import glob
import json
import os
import sys

STEP_KERNELS = ("k_arn_a1", "k_arn_a2", "k_arn_d1", "k_reduce", "k_red_d1", "k_post", "k_lan_", "k_spmv_mf", "k_ilv")
GATHER_KERNELS = ("k_spmv_mf",)


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            per.setdefault(name, 0.0)
            per[name] += float(r["Counter_Value"])
    return per


def main():
    fdir, wdir, cfg, ngpu, K, out = sys.argv[1:7]
    K = int(K)
    ff = float(os.environ.get("FETCH_FACTOR", "2"))
    fetch = load(fdir, "FETCH_SIZE")
    write = load(wdir, "WRITE_SIZE")
    # the doubling applies to wide streaming reads; k_spmv_mf's random 64-byte gathers are
    # tallied at their size (raw FETCH_SIZE = 64 B x nonzeros at C3)
    step_f = sum(v * (1.0 / ff if any(g in k for g in GATHER_KERNELS) else 1.0)
                 for k, v in fetch.items() if any(s in k for s in STEP_KERNELS))
    step_w = sum(v for k, v in write.items() if any(s in k for s in STEP_KERNELS))
    per_kernel = {k: {"fetch_KiB": fetch.get(k, 0.0), "write_KiB": write.get(k, 0.0)}
                  for k in sorted(set(fetch) | set(write))}
    res = {"config": cfg, "n_gpus": int(ngpu), "K": K, "fetch_factor": ff,
           "fetch_factor_note": "x%g on streaming reads; x1 on the random 64-B gathers of %s" % (ff, GATHER_KERNELS),
           "hbm_bytes_per_step": (ff * step_f + step_w) * 1024.0 / K,
           "fetch_bytes_per_step_raw": step_f * 1024.0 / K, "write_bytes_per_step": step_w * 1024.0 / K,
           "per_kernel_KiB": per_kernel}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_kernel_KiB"}))


if __name__ == "__main__":
    main()
