"""The pt_ss_k job solver's exactness arguments, checked on the CPU (no GPU).

ss_sca_rel_red_body (shyft_amd/csrc/device/ptssk_dev.h) departs from the sequential bisection of
boost::math::tools::bisect (skaugen.h:57-82, restated in oracle/src/ptssk.hpp) in three ways that must not move a bit:
the grouped rounds (the midpoints of the next 2 or 3 levels at once, then the sequential loop replayed over them),
the midpoint sign without the pdfs' divisions where it is certain, and (r06) the sign from the pdfs' exp arguments
where they decide it. tools/mb/ptssk_group_emu.cpp replays all of them against the oracle's bisect and counts every
disagreement; here it runs on 4,000 recorded jobs of the bench region's year (tests/golden/ptssk_jobs_sample.npy,
written by tools/mb/ptssk_jobs -o from the oracle, 1,500 of them from the nu_a band in [1024, 4096) where the exp
arguments do not decide and the full path runs). The year's 1,031,709 jobs: profiles/r06/ptssk_group_emu_expskip.txt.
"""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_job_solver_shortcuts_reproduce_the_oracle_bisection(tmp_path):
    exe = tmp_path / "ptssk_group_emu"
    subprocess.run(["g++", "-O2", "-std=c++17", "-mfma", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tools", "mb", "ptssk_group_emu.cpp")], check=True, cwd=ROOT, timeout=300)
    jobs = np.load(os.path.join(ROOT, "tests", "golden", "ptssk_jobs_sample.npy"))
    assert jobs.shape == (4000, 9) and jobs.dtype == np.float64
    binf = tmp_path / "jobs.bin"
    jobs.tofile(binf)
    p = subprocess.run([str(exe), str(binf)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    m = re.search(r"bisections checked (\d+): differing brackets: sign surrogate (\d+), D=2 (\d+), D=3 (\d+)", p.stdout)
    assert m, p.stdout
    checked, bad_sign, bad2, bad3 = map(int, m.groups())
    assert checked == 4000 and bad_sign == 0 and bad2 == 0 and bad3 == 0
    m = re.search(r"decided by the exp arguments (\d+) \(differing from the exps' decision: (\d+)\)", p.stdout)
    assert m and int(m.group(1)) > 0 and int(m.group(2)) == 0, p.stdout
