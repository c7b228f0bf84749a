"""Per-kernel-class MFMA / VALU busy and effective clock from a rocprofv3 --pmc pass.

Counters (one pass, tools/gpu.sh pmc): SQ_VALU_MFMA_BUSY_CYCLES (per-SIMD cycles the matrix
pipe is busy, summed over SIMDs), SQ_ACTIVE_INST_VALU (quad-cycles, summed over CUs... per the
VALUBusy formula), GRBM_GUI_ACTIVE (GPU-busy cycles; rocprofv3 reports the sum over the 8 XCDs),
SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY (wave-state split).

  MfmaUtil  = MFMA_BUSY / (GUI_ACTIVE/8 * 1024 SIMDs)          (rocprofv3 derived 'MfmaUtil')
  VALUBusy  = ACTIVE_INST_VALU / 256 CUs / (GUI_ACTIVE/8)        (rocprofv3 derived 'VALUBusy')
  clock     = GUI_ACTIVE/8 / kernel duration                      (MI355X_MICROARCH.md, DVFS give-back)
  LDS pass (optional): lds_idx_active_per_cu_cycle = SQ_LDS_IDX_ACTIVE / 256 / (GUI_ACTIVE/8),
  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, wait_inst_lds_frac = SQ_WAIT_INST_LDS /
  SQ_WAVE_CYCLES (issue stalls on the LDS queue), lds_insts = SQ_INSTS_LDS
  memory pass (optional): ta_busy_per_cu = TA_TA_BUSY_sum / 256 / (GUI_ACTIVE/8), l2_hit_rate = TCC_HIT / (HIT + MISS),
  sq_inst_level_vmem_frac = SQ_INST_LEVEL_VMEM / SQ_WAVE_CYCLES (average VMEM instructions in flight per wave)

usage: python tools/pmc_busy.py <counter_collection.csv> <out.json> [label]
"""
import collections
import csv
import json
import sys

CLASSES = [("conv_gemm_kernel", "conv_gemm (1x1 / implicit-GEMM, split-bf16 MFMA)"),
           ("gemm_res_kernel", "conv_gemm (1x1 / implicit-GEMM, split-bf16 MFMA)"),
           ("gemm_chunk_kernel", "conv_gemm (1x1 / implicit-GEMM, split-bf16 MFMA)"),
           ("gemm_attn_in_kernel", "conv_gemm (1x1 / implicit-GEMM, split-bf16 MFMA)"),
           ("dwconv_gram", "dwconv_gram (MDTA pass 1: dwconv + MFMA Gram)"),
           ("ffn_fused_kernel<96>", "ffn_fused C96 (LN + project_in + gate + project_out)"),
           ("ffn_fused_kernel<48>", "ffn_fused C48 (LN + project_in + gate + project_out)"),
           ("gdfn_out_kernel", "gdfn_out (fused GDFN tail: dwconv + gate + MFMA project_out)"),
           ("gdfn2_kernel", "gdfn_out (fused GDFN tail: dwconv + gate + MFMA project_out)"),
           ("dwconv_gate_kernel", "dwconv_gate (unfused GDFN gate, C >= 192)"),
           ("conv_small", "conv_small (stem / head convs)"),
           ("mfma_loop", "mfma_peak micro (bare MFMA loop)")]


def cls_of(name):
    for p, lab in CLASSES:
        if p in name:
            return lab
    return "other"


def main():
    path, out = sys.argv[1:3]
    label = sys.argv[3] if len(sys.argv) > 3 else ""
    disp = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kdlae::", "")
        dur = None
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        meta[key] = (name, dur)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for key, c in disp.items():
        name, dur = meta[key]
        a = agg[cls_of(name)]
        a["dispatches"] += 1
        for k, v in c.items():
            a[k] += v
        if dur:
            a["seconds"] += dur
    res = {"label": label, "source": path, "formulas": __doc__.split("usage")[0].strip(), "classes": {}}
    for lab, a in sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        gui = a.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        row = {"dispatches": int(a["dispatches"])}
        if gui > 0:
            if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
                row["mfma_util"] = round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * 1024), 4)
            if "SQ_ACTIVE_INST_VALU" in a:
                row["valu_busy"] = round(a["SQ_ACTIVE_INST_VALU"] / 256 / gui, 4)
            if a.get("seconds"):
                row["clock_ghz"] = round(gui / a["seconds"] / 1e9, 3)
                row["seconds"] = round(a["seconds"], 6)
            if "SQ_LDS_IDX_ACTIVE" in a:
                row["lds_idx_active_per_cu_cycle"] = round(a["SQ_LDS_IDX_ACTIVE"] / 256 / gui, 4)
                if a["SQ_LDS_IDX_ACTIVE"]:
                    row["lds_bank_conflict_frac"] = round(a.get("SQ_LDS_BANK_CONFLICT", 0.0) / a["SQ_LDS_IDX_ACTIVE"], 4)
            if "TA_TA_BUSY_sum" in a:
                row["ta_busy_per_cu"] = round(a["TA_TA_BUSY_sum"] / 256 / gui, 4)
            if "TCC_HIT_sum" in a and (a["TCC_HIT_sum"] + a.get("TCC_MISS_sum", 0.0)) > 0:
                row["l2_hit_rate"] = round(a["TCC_HIT_sum"] / (a["TCC_HIT_sum"] + a.get("TCC_MISS_sum", 0.0)), 4)
        wc = a.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_INST_LEVEL_VMEM"):
                if k in a:
                    row[k.lower() + "_frac_of_wave_cycles"] = round(a[k] / wc, 4)
        row["raw"] = {k: v for k, v in a.items() if k not in ("dispatches",)}
        res["classes"][lab] = row
    json.dump(res, open(out, "w"), indent=1)
    for lab, row in res["classes"].items():
        print(f"{lab:60s} n={row['dispatches']:5d} mfma={row.get('mfma_util')} valu={row.get('valu_busy')} "
              f"clk={row.get('clock_ghz')} lds={row.get('lds_idx_active_per_cu_cycle')} "
              f"bankc={row.get('lds_bank_conflict_frac')} waitlds={row.get('sq_wait_inst_lds_frac_of_wave_cycles')} "
              f"ta={row.get('ta_busy_per_cu')} l2hit={row.get('l2_hit_rate')} "
              f"wait={row.get('sq_wait_any_frac_of_wave_cycles')} winst={row.get('sq_wait_inst_any_frac_of_wave_cycles')} "
              f"vmemlvl={row.get('sq_inst_level_vmem_frac_of_wave_cycles')}")


if __name__ == "__main__":
    main()
