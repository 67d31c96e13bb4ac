"""The committed measurement evidence is self-consistent (CPU only): the bench line's roofline `frac` is
reproduced from the rocprofv3 kernel trace of the same bench.py run (tools/trace_roofline.py), and the line keeps
the bench.py contract's fields (task's measurement rules)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FINAL = os.path.join(ROOT, "profiles", "r6", "final")


def _line(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_bench_line_fields():
    d = _line(os.path.join(FINAL, "bench.json"))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-4
    # achieved = algorithmic bytes per launch over the event-timed mean launch
    assert abs(r["achieved"] - r["alg_bytes_per_launch"] / (r["avg_launch_ms"] * 1e-3) / 1e9) / r["achieved"] < 1e-3
    # value is the samples of one step over the step time
    assert d["value"] > 0 and d["ms_per_step"] > 0
    c = d["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0


def test_trace_reproduces_frac():
    bp = os.path.join(FINAL, "benchprof")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_roofline.py"),
                          os.path.join(bp, "bp_kernel_trace.csv"), os.path.join(bp, "bench_under_rocprof.json")],
                         check=True, capture_output=True, text=True).stdout
    got = json.loads(out)
    assert got["statistics_frame_dispatches"] > 0
    # the line's HIP-event mean and the profiler's mean of the same dispatches agree within a few per cent
    assert abs(got["frac_rel_diff"]) < 0.05, got
    committed = _line(os.path.join(bp, "trace_roofline.json"))
    assert committed["trace_frac"] == got["trace_frac"]
