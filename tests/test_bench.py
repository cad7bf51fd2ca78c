"""The bench.py contract (the driver's BENCH line): one JSON line with the metric, the whole-job
value, the timing fields, and the roofline and cpu_baseline objects, on the headline workload."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_line_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--cpu-seconds", "2"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "roofline_shade", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["config"]["workload"].startswith("C3: synth-1M, 1024x1024, 64 spp")
    # value = traced rays per second over the timed steps; the reference-equivalent count beside it
    assert abs(d["value"] - d["rays_traced_per_path"] * 1024 * 1024 * 64 / (d["ms_per_step"] * 1e-3) / 1e6) < 0.01 * d["value"]
    assert d["value"] == d["mrays_traced_per_s"]
    assert abs(d["mrays_reference_equivalent_per_s"] - d["rays_per_path"] * 1024 * 1024 * 64
               / (d["ms_per_step"] * 1e-3) / 1e6) < 0.01 * d["value"]
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert 0.25 < rf["frac"] <= 1.05 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 0.01
    assert rf["peak"] == 34500.0 and rf["unit"] == "GB/s"  # a hardware peak (MI355X aggregate L2)
    # the drop-in frame loop: 1-spp calls, films bit-identical to the batched render
    di = d["dropin"]
    for pol in ("queued", "sync", "sync_read"):
        assert di[pol]["film_equals_batched"] is True and di[pol]["ms_per_frame"] > 0, pol
    assert di["queued"]["ms_per_frame"] <= di["sync_read"]["ms_per_frame"]
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] in ("reference", "port") and cb["value"] > 0
