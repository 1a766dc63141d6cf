"""bench.py's stdout is its one JSON line: native code that prints on descriptor 1 (RCCL's version banner
when the communicator is created) goes to stderr once bench.json_stdout() has run."""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

SCRIPT = r"""
import ctypes, os, sys
sys.path.insert(0, sys.argv[1])
import bench
out = bench.json_stdout()
print("python noise")                      # sys.stdout -> descriptor 1 -> stderr
os.write(1, b"native noise\n")             # what a C library writes on descriptor 1
ctypes.CDLL(None).puts(b"libc puts noise")  # buffered C stdio on descriptor 1
ctypes.CDLL(None).fflush(None)
print('{"metric": "m", "value": 1}', file=out, flush=True)
"""


def test_bench_stdout_is_the_json_line_only():
    p = subprocess.run([sys.executable, "-c", SCRIPT, str(ROOT)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    assert json.loads(lines[0])["value"] == 1
    assert "python noise" in p.stderr and "native noise" in p.stderr and "libc puts noise" in p.stderr
