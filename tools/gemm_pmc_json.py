"""profiles/<tag>_gemm_mfma_busy.json from a tools/gemm_planes_pmc.sh summary table
(the per-shape averages of the six C3 GEMMs' counters):

    python tools/gemm_pmc_json.py gpurun_out/gemm_pmc/summary.txt profiles/r03_gemm_mfma_busy.json
"""
import json
import sys

rows = {}
lines = open(sys.argv[1]).read().split("\n")
shapes = lines[0].split()[1:]
for ln in lines[1:]:
    if ln.strip():
        f = ln.split()
        rows[f[0]] = dict(zip(shapes, map(float, f[1:])))
out = {"source": "tools/gemm_planes_pmc.sh (rocprofv3 --pmc passes over the six C3 MLP GEMMs, "
                 "standalone, 10 launches each)",
       "definition": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 "
                     "XCDs): the fraction of SIMD-cycles the matrix pipe was busy; hbm_bytes = "
                     "FETCH_SIZE x 2 (gfx950) + WRITE_SIZE, KiB -> bytes",
       "shapes": {}}
for s in shapes:
    g = rows["GRBM_GUI_ACTIVE"][s]
    out["shapes"][s] = {
        "mfma_busy": rows["SQ_VALU_MFMA_BUSY_CYCLES"][s] / (1024 * g / 8),
        "mfma_busy_cycles": rows["SQ_VALU_MFMA_BUSY_CYCLES"][s],
        "grbm_gui_active": g,
        "lds_bank_conflict": rows["SQ_LDS_BANK_CONFLICT"][s],
        "wait_any_frac": rows["SQ_WAIT_ANY"][s] / rows["SQ_WAVE_CYCLES"][s],
        "wait_inst_any_frac": rows["SQ_WAIT_INST_ANY"][s] / rows["SQ_WAVE_CYCLES"][s],
        "hbm_bytes": (rows["FETCH_SIZE"][s] * 2 + rows["WRITE_SIZE"][s]) * 1024,
    }
open(sys.argv[2], "w").write(json.dumps(out, indent=1))
print({s: round(v["mfma_busy"], 3) for s, v in out["shapes"].items()},
      {s: round(v["hbm_bytes"] / 1e6, 1) for s, v in out["shapes"].items()})
