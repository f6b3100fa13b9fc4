"""csrc/acos_cr.h (the literal light chain's acos, Mylight.cpp:375-396) on the host: built with g++ and
compared with mpmath's correctly rounded acos over [-1, 1] (uniform, near -1, 0 and 1, and special
values), also when its libm start value is moved 1-2 ulp (ocml's acos is within 1 ulp).  Correct
rounding is what makes the GPU's literal chain reproduce the oracle's glibc angles wherever glibc
itself is correctly rounded."""
import subprocess
import sys

from conftest import ROOT


def test_acos_cr_is_correctly_rounded():
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "acos_cr_check.py"), "20000"], capture_output=True,
                       text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "acos_cr     differs from correctly rounded on 0 of" in r.stdout
