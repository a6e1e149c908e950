"""The committed bench line (profiles/r1h_bench_quad13.json, written by bench.py on an MI355X)
keeps the bench.py JSON contract: required keys, whole-job value consistent with the step time,
roofline fraction = achieved / peak, and a CPU baseline entry. CPU-only: reads a committed file."""
import json
import math
import pathlib

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
LINE = ROOT / "profiles" / "r1h_bench_quad13.json"

REQUIRED = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]


@pytest.fixture(scope="module")
def line():
    if not LINE.exists():
        pytest.skip("no committed bench line")
    return json.loads(LINE.read_text().strip().splitlines()[-1])


def test_required_keys(line):
    for k in REQUIRED:
        assert k in line, k
    assert line["higher_is_better"] is True
    assert line["scaling"] == "weak"
    assert line["dtype"] == "f64"
    assert "workload" in line["config"]


def test_value_matches_step_time(line):
    # value = instances processed per second over all ranks = batch_per_gpu * n_gpus / step time
    b = line["config"]["batch_per_gpu"] * line["n_gpus"]
    assert math.isclose(line["value"], b / (line["ms_per_step"] * 1e-3), rel_tol=1e-6)


def test_roofline_fraction(line):
    r = line["roofline"]
    assert r["unit"] in ("GB/s", "TFLOP/s") and r["bound"] in ("hbm", "mfma", "valu_fp64", "valu_fp32")
    assert math.isclose(r["frac"], r["achieved"] / r["peak"], rel_tol=1e-9)
    # achieved = algorithmic flops per launch / kernel duration
    assert math.isclose(r["achieved"], r["flops_per_launch"] / (r["kernel_ms"] * 1e-3) / 1e12, rel_tol=1e-6)
    assert 0.0 < r["frac"] <= 1.0


def test_cpu_baseline(line):
    c = line["cpu_baseline"]
    assert c["kind"] in ("port", "reference")
    assert c["cores"] >= 1 and c["value"] > 0 and c["sample"]


def test_bench_refuses_world_size_mismatch():
    """A launcher's WORLD_SIZE that differs from --gpus is refused before any GPU work (exit 2, nothing
    on stdout), so a driver run can never report the wrong number of GPUs."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4"], env=env,
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 2 and out.stdout == ""
    assert "differs from --gpus 4" in out.stderr
