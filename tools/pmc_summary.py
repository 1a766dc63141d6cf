"""Summarise rocprofv3 --pmc passes written by tools/pmc.sh.

usage: python tools/pmc_summary.py <pmc root dir> <config name> [--json profiles/pmc_traffic.json]
                                   [--skip N] [--deep-json out.json "note"] [--levels]

--skip N drops each kernel's first N dispatches of every profiled run (the warm-up frames: before the
background-store-elision masks settle, frames 0-1 store every background pixel), so the averages are
steady-state.  --deep-json writes every counter per wave (SQ cycle counters in quad-cycles) per kernel.

Prints per-kernel averages (per dispatch) of every collected counter plus derived figures, and
with --json merges {config: {kernel: {...}}} into the traffic file bench.py reads.

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads, so
hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.  (Exact for 16-B-per-lane loads; our
8-B texel and 4-B plane loads are uncalibrated, which the JSON states.)
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

SHORT = {  # mangled and demangled spellings
    "k_gbuffer": "gbuffer", "k_albedo": "full_screen_albedo",
    "k_direct_fused": "direct_lit_emissive", "k_direct_lit_w4": "direct_lit",
    "k_directILb0ELb1": "direct_lit", "k_direct<false, true": "direct_lit",
    "k_directILb1ELb0": "direct_emissive", "k_direct<true, false": "direct_emissive",
    "k_indirectILb0": "indirect_lit_ambient", "k_indirect<false": "indirect_lit_ambient",
    "k_indirectILb1": "indirect_multiple_bounces", "k_indirect<true": "indirect_multiple_bounces",
    "k_spatialILb0": "indirect_spatial_reuse", "k_spatial<false": "indirect_spatial_reuse",
    "k_spatialILb1": "emissive_spatial_reuse", "k_spatial<true": "emissive_spatial_reuse",
    "k_wf_": "indirect_wavefront", "k_demod3": "demodulation", "k_denoise3": "denoise", "k_tone": "tone_mapping", "k_trace": "trace",
    "k_f16": "f16_selftest", "k_build_wide": "scene_build_wide", "k_fill_blas_leaves": "scene_fill_leaves",
    "k_fill_tlas_leaves": "scene_fill_leaves", "k_collapse_decide": "scene_collapse_leaves",
    "k_collapse_write": "scene_collapse_leaves",
}


LEVELS = "--levels" in sys.argv  # the a-trous levels per level (denoise_L0..L3) instead of one "denoise" row


def short(name: str) -> str:
    if LEVELS and "k_denoise3" in name:
        m = re.search(r"k_denoise3(?:<\d+, (\d)>|ILi\dELi(\d)E)", name)
        if m:
            return f"denoise_L{m.group(1) or m.group(2)}"
    for k, v in SHORT.items():
        if k in name:
            return v
    return name[:40]


def load(root: Path, skip: int = 0):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    dur = defaultdict(list)
    for f in sorted(root.glob("**/*counter_collection.csv")):
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if not k or k.startswith("__amd"):
                    continue
                d = int(row["Dispatch_Id"])
                per[d][row["Counter_Name"]] += float(row["Counter_Value"])
                names[d] = k
        seen = defaultdict(int)
        for d in sorted(per):
            seen[names[d]] += 1
            if seen[names[d]] <= skip:
                continue
            for c, v in per[d].items():
                vals[names[d]][c].append(v)
    for f in sorted(root.glob("**/*kernel_trace.csv")):
        seen = defaultdict(int)
        with open(f) as fh:
            rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Start_Timestamp"]))
        for row in rows:
            k = short(row["Kernel_Name"])
            seen[k] += 1
            if seen[k] > skip:
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    return vals, dur


def summarise(vals, dur):
    out = {}
    for k, cs in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"counters": {c: round(v, 1) for c, v in avg.items()}}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["hbm_bytes_per_launch"] = int(2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024)
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            t = avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]
            e["l2_hit"] = round(avg["TCC_HIT_sum"] / t, 3) if t else None
        if avg.get("SQ_WAVES"):
            w = avg["SQ_WAVES"]
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if c in avg:
                    e[c.replace("SQ_INSTS_", "").lower() + "_per_wave"] = round(avg[c] / w, 1)
        if avg.get("SQ_BUSY_CYCLES") and "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
            e["valu_active_frac_of_wave_cycles"] = round(avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"], 3)
        if dur.get(k):
            e["avg_ms_profiled"] = round(sum(dur[k]) / len(dur[k]), 4)
        out[k] = e
    return out


def deep(vals, dur):
    out = {}
    for k, cs in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        w = avg.get("SQ_WAVES")
        if not w:
            continue
        e = {"per_wave": {c: round(v / w, 1) if c != "SQ_WAVES" else 1.0 for c, v in sorted(avg.items())},
             "waves_per_launch": round(w, 1)}
        if dur.get(k):
            e["avg_ms_profiled"] = round(sum(dur[k]) / len(dur[k]), 4)
        out[k] = e
    return out


def main():
    root, config = Path(sys.argv[1]), sys.argv[2]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    vals, dur = load(root, skip)
    s = summarise(vals, dur)
    if "--deep-json" in sys.argv:
        i = sys.argv.index("--deep-json")
        Path(sys.argv[i + 1]).write_text(json.dumps({"note": sys.argv[i + 2], "config": config, "skip": skip,
                                                     "kernels": deep(vals, dur)}, indent=1))
    for k, e in sorted(s.items()):
        extra = {x: y for x, y in e.items() if x != "counters"}
        print(f"{k:28s} {extra}")
    if "--json" in sys.argv:
        p = Path(sys.argv[sys.argv.index("--json") + 1])
        d = json.loads(p.read_text()) if p.exists() else {}
        d.setdefault("note", "rocprofv3 --pmc (kernel-trace only), FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md "
                             "HBM section); x2 exact for 16-B/lane reads, 4/8-B texel reads uncalibrated")
        d.setdefault("configs", {})[config] = {"kernels": s, "skipped_warmup_dispatches": skip}
        p.write_text(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
