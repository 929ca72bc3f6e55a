"""The config-E sweep's binary64 LeastAllocated form (ms_kernels.hip la_r /
la_a / eval_fast) equals the reference's integer leastRequestedScore on every
boundary case tests/c/la_f64_exact.c generates (CPU; the GPU parity suite runs
the kernel itself, tests/test_gpu_parity.py::test_resource_sequential_capacity_forms)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_la_f64_exact(tmp_path):
    exe = tmp_path / "la_f64_exact"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(HERE, "c", "la_f64_exact.c"), "-lm", "-o",
                    str(exe)], check=True)
    out = subprocess.run([str(exe), "5000000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    assert "mismatches=0" in out.stdout
