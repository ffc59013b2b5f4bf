"""cf_per_kw (the kernels' gen_per_kw = cf / 1e6 without a per-hour division)
is the IEEE quotient for every integer |cf| <= 2e7: exhaustive C check with
the host's fma (IEEE, like the device's v_fma_f64)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fma_corrected_division_is_exact(tmp_path):
    exe = tmp_path / "check_cf_div"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(HERE, "check_cf_div.c"), "-lm"], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert int(out.strip()) == 0
