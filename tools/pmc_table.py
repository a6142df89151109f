"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel dispatch:
effective clock, MFMA busy fraction, wave-cycle breakdown, LDS stalls."""
import collections
import csv
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
last_n = int(sys.argv[3]) if len(sys.argv) > 3 else 0
d = collections.OrderedDict()
for r in csv.DictReader(open(path)):
    key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
    e = d.setdefault(key, {"grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]),
                           "lds": int(r["LDS_Block_Size"]), "vgpr": int(r["VGPR_Count"]),
                           "agpr": int(r["Accum_VGPR_Count"])})
    e[r["Counter_Name"]] = float(r["Counter_Value"])
    e["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
items = [(k, v) for k, v in d.items() if pat in k[1]]
if last_n:
    items = items[-last_n:]
for (i, k), v in items:
    g = v.get("GRBM_GUI_ACTIVE", 0)
    clk = g / 8 / v["dur"] / 1e9 if v["dur"] else 0
    mf = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * g / 8) if g else 0
    w = v.get("SQ_WAVE_CYCLES", 1) or 1
    name = k.split("(")[0].replace("void ", "").replace("ainp::", "")[:48]
    print(f"{i:4d} {name:48s} {v['dur'] * 1e3:7.3f}ms {clk:4.2f}GHz mfma {mf:5.3f} "
          f"wait {v.get('SQ_WAIT_ANY', 0) / w:4.2f} winst {v.get('SQ_WAIT_INST_ANY', 0) / w:4.2f} "
          f"act {v.get('SQ_ACTIVE_INST_ANY', 0) / w:4.2f} wlds {v.get('SQ_WAIT_INST_LDS', 0) / w:4.2f} "
          f"bconf/cyc {v.get('SQ_LDS_BANK_CONFLICT', 0) / (g / 8 * 256) if g else 0:5.3f} "
          f"v{v['vgpr']}/a{v['agpr']} lds{v['lds']}")
