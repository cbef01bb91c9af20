"""Merge rocprofv3 --pmc counter-collection CSVs (separate passes over the same
command) into per-kernel means with derived figures:

  SQ counters are summed over the chip; SQ_*_CYCLES / SQ_ACTIVE_* / SQ_WAIT_*
  count quad-cycles (4 clocks) per wave; GRBM_GUI_ACTIVE counts clocks summed
  over the 8 XCDs.  Derived (per launch):
    duration_us        = GRBM_GUI_ACTIVE / 8 / 2400 MHz (the launch's busy clocks at the peak clock)
    valu_per_wave      = SQ_INSTS_VALU / SQ_WAVES
    waves_per_simd     = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8) / 1024 SIMDs (mean resident waves)
    valu_issue_share   = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of a wave's life issuing VALU)
    wait_inst_share    = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (waiting for an issue slot / dependency)
    wait_any_share     = SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked at s_waitcnt / barrier)
    simd_valu_busy     = 4 * SQ_ACTIVE_INST_VALU * 2 / (GRBM_GUI_ACTIVE / 8 * 1024): VALU cycles per SIMD cycle
                         (wave64 issues over 2 cycles on the 32-lane gfx950 SIMD; approximate)
  usage: pmc_sq_json.py OUT.json pass1.csv [pass2.csv ...]"""
import collections
import csv
import json
import sys


def main():
    out, paths = sys.argv[1], sys.argv[2:]
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for row in csv.DictReader(open(p)):
            d[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {"note": __doc__.strip().splitlines()[0], "derivation": __doc__.split("Derived (per launch):")[1].split("usage")[0].strip(),
           "kernels": {}}
    for k, ctr in d.items():
        m = {c: sum(v) / len(v) for c, v in ctr.items()}
        n = {c: len(v) for c, v in ctr.items()}
        e = {"launches": max(n.values()), "mean": m}
        g = m.get("GRBM_GUI_ACTIVE")
        w = m.get("SQ_WAVES")
        wc = m.get("SQ_WAVE_CYCLES")
        der = {}
        if g:
            der["duration_us"] = g / 8 / 2400.0
        if w and m.get("SQ_INSTS_VALU") is not None:
            der["valu_per_wave"] = m["SQ_INSTS_VALU"] / w
        if w and m.get("SQ_INSTS_LDS") is not None:
            der["lds_per_wave"] = m["SQ_INSTS_LDS"] / w
        if wc and g:
            der["waves_per_simd"] = 4 * wc / (g / 8) / 1024
        if wc:
            for key, c in (("valu_issue_share", "SQ_ACTIVE_INST_VALU"), ("wait_inst_share", "SQ_WAIT_INST_ANY"),
                           ("wait_any_share", "SQ_WAIT_ANY"), ("any_issue_share", "SQ_ACTIVE_INST_ANY"),
                           ("lds_issue_share", "SQ_ACTIVE_INST_LDS")):
                if m.get(c) is not None:
                    der[key] = m[c] / wc
        if g and m.get("SQ_ACTIVE_INST_VALU") is not None:
            der["simd_valu_busy"] = 4 * m["SQ_ACTIVE_INST_VALU"] * 2 / (g / 8 * 1024)
        if g and m.get("SQ_LDS_IDX_ACTIVE") is not None:
            der["lds_idx_active_per_cu_cycle"] = 4 * m["SQ_LDS_IDX_ACTIVE"] / (g / 8 * 256)
        e["derived"] = der
        res["kernels"][k] = e
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
