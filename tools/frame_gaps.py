"""GPU idle time between the kernels of consecutive frames, from a rocprofv3 kernel trace.

usage: python tools/frame_gaps.py <run_kernel_trace.csv> <first-kernel-of-frame substring> [skip frames]

Frames are cut at each launch of the named kernel (e.g. k_gbuffer).  Per frame: the span from its first
kernel's start to the next frame's first start, the time at least one kernel ran (union of intervals),
and the idle rest (launch latency, cross-stream dependency waits, host enqueue stalls)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark, skip = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 5
starts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
spans, busy, kernels = [], [], []
for a, b in zip(starts[skip:], starts[skip + 1:]):
    t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    iv = sorted((int(r["Start_Timestamp"]), min(int(r["End_Timestamp"]), t1)) for r in rows[a:b])
    u, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                u += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    u += cur_e - cur_s
    spans.append((t1 - t0) / 1e3)
    busy.append(u / 1e3)
    kernels.append(b - a)
print(f"frames {len(spans)}: span {statistics.median(spans):.1f} us, busy {statistics.median(busy):.1f} us, "
      f"idle {statistics.median(spans) - statistics.median(busy):.1f} us, kernels/frame {statistics.median(kernels)}")
