"""Lane efficiency inside spatial reuse's neighbour loop (instrumented builds exp_lanestats/sp{0,1,2}.so:
-DHK_LANE_STATS -DHK_SP_STATS=k ticks per neighbour iteration (0), at the occlusion march (1) and at
the merge (2)).  usage: HK_LIB=exp_lanestats/spK.so python tools/spatial_lanes.py"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from lane_stats import measure  # noqa: E402

out = {}
for cfg in ("scene-1080p-full", "city-4k"):
    d = measure(cfg, False)
    out[cfg] = d.get("indirect_spatial_reuse")
print(json.dumps(out))
