"""Where the timed region of a short bench run goes, from a rocprofv3 kernel trace of `bench.py --steps K --warmup W`.

usage: python tools/timed_span.py <run_kernel_trace.csv> <warmup> <steps> [first-kernel-of-frame substring]

Frames are cut at each launch of the named kernel (default k_gbuffer); frame f = the f-th cut.  Prints the idle gap
before the first timed frame's first kernel, the GPU span of the timed frames (first timed kernel start to last
timed kernel end), the per-frame spans inside it, and how far the span exceeds K x the median steady-state span
(the fill / drain cost a short timed region pays)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
W, K = int(sys.argv[2]), int(sys.argv[3])
mark = sys.argv[4] if len(sys.argv) > 4 else "k_gbuffer"
cuts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
cuts.append(len(rows))


def frame(f):
    return rows[cuts[f]:cuts[f + 1]]


def start(f):
    return min(int(r["Start_Timestamp"]) for r in frame(f))


def end(f):
    return max(int(r["End_Timestamp"]) for r in frame(f))


gap = (start(W) - end(W - 1)) / 1e3
span = (end(W + K - 1) - start(W)) / 1e3
per = [(start(f + 1) - start(f)) / 1e3 for f in range(W, W + K - 1)]
steady = statistics.median(per)
print(f"idle before the first timed frame: {gap:.1f} us")
print(f"timed frames {W}..{W + K - 1}: GPU span {span:.1f} us = {span / K:.4f} ms/frame; steady frame {steady:.1f} us")
print(f"frame-to-frame spans (us): " + " ".join(f"{p:.0f}" for p in per))
print(f"last timed frame: first kernel start to last kernel end {(end(W + K - 1) - start(W + K - 1)) / 1e3:.1f} us")
print(f"span - K x steady = {span - K * steady:.1f} us")
for f in (W, W + 1, W + K - 1):
    print(f"frame {f}:", " ".join(f"{r['Kernel_Name'].split('(')[0].split('<')[0]}@{(int(r['Start_Timestamp']) - start(W)) / 1e3:.0f}"
                                 f"+{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.0f}" for r in frame(f)))
