"""The VALU issue bound of the traversal kernels, from a rocprofv3 --pmc pass with SQ_WAVES and SQ_INSTS_VALU (every
kernel alone: tools/pmc_deep.sh's isolation options).

A wave64 VALU instruction occupies its SIMD's vector issue for 4 cycles (MI355X_MICROARCH.md, 'vector-instruction
ISSUE cost'; v_rcp / v_sqrt / v_exp 8: SQ_INSTS_VALU_TRANS_F32 counts those), so a launch needs at least
  t_valu = (SQ_INSTS_VALU + SQ_INSTS_VALU_TRANS_F32) x 4 cycles / (1024 SIMDs x f_clk)
of vector issue, whatever its memory traffic.  valu_frac = t_valu / the launch's measured duration is the fraction of
the chip's vector issue capacity the launch fills: near 1 it is bound by its instruction count, not by HBM (the
traversal kernels' HBM fraction is 0.1-0.3).  f_clk: 2.4 GHz (the peak engine clock; under load the chip runs lower,
MI355X_MICROARCH.md 'DVFS give-back', so the fraction is a lower bound).

usage: python tools/valu_summary.py <pmc run dir> <config> [--json profiles/valu_issue.json] [--skip N]"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import short  # noqa: E402

CLK_GHZ, SIMDS = 2.4, 1024


def main():
    root, config = Path(sys.argv[1]), sys.argv[2]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 2
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for f in sorted(root.glob("**/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            d = (str(f), r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[d] = (short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    by = defaultdict(list)
    for d, c in per.items():
        by[meta[d][0]].append((c, meta[d][1]))
    out = {}
    for k, rows in sorted(by.items()):
        rows = rows[skip:] if len(rows) > skip + 1 else rows
        n = len(rows)
        valu = sum(c.get("SQ_INSTS_VALU", 0.0) for c, _ in rows) / n
        trans = sum(c.get("SQ_INSTS_VALU_TRANS_F32", 0.0) for c, _ in rows) / n
        waves = sum(c.get("SQ_WAVES", 0.0) for c, _ in rows) / n
        ms = sum(t for _, t in rows) / n
        if not valu or not waves:
            continue
        t_valu = (valu + trans) * 4 / (SIMDS * CLK_GHZ * 1e9) * 1e3
        out[k] = {"valu_per_launch": int(valu), "valu_per_wave": round(valu / waves, 1), "waves": int(waves),
                  "t_valu_ms": round(t_valu, 4), "profiled_ms": round(ms, 4), "valu_frac": round(t_valu / ms, 3),
                  "dispatches": n}
        print(f"{k:28s} VALU/wave {valu / waves:8.1f}  VALU-issue floor {t_valu:.4f} ms  profiled {ms:.4f} ms  "
              f"frac {t_valu / ms:.3f}")
    if "--json" in sys.argv:
        p = Path(sys.argv[sys.argv.index("--json") + 1])
        d = json.loads(p.read_text()) if p.exists() else {"note": __doc__.split("\n\n")[1].replace("\n", " "),
                                                           "clock_ghz": CLK_GHZ, "simds": SIMDS, "configs": {}}
        d["configs"][config] = {"source": str(root), "kernels": out}
        p.write_text(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
