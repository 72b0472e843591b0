"""bench.py uses a committed PMC summary only for the library it measured: the summary's
lib_sha256 must equal the sha256 of the library the bench process loads, else `traffic` is null and the reason names
both builds. CPU only (no HIP call: lib_sha hashes the file)."""
import json
import re
import types
from pathlib import Path

import pytest

import bench
from shyft_amd import _native

ROOT = Path(__file__).resolve().parents[1]


def _args(**kw):
    a = dict(stack="pt_gs_k", idw=False, btk=False, chunk=438, steps=20, warmup=5, shards=1)
    a.update(kw)
    return types.SimpleNamespace(**a)


@pytest.fixture
def tree(tmp_path, monkeypatch):
    prof = tmp_path / "profiles" / "rXX"
    prof.mkdir(parents=True)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "PROFILE_DIR", str(prof))
    monkeypatch.setattr(_native, "lib_sha", lambda path=None: "ab" * 32)
    return prof


def test_no_summary(tree):
    d, why = bench.pmc_summary(_args(), 1 << 20)
    assert d is None and "no PMC summary" in why


def test_summary_of_another_build_is_refused(tree):
    a = _args()
    (tree / f"pmc_{bench.workload_tag(a, 1 << 20)}.json").write_text(json.dumps({"lib_sha256": "cd" * 32}))
    d, why = bench.pmc_summary(a, 1 << 20)
    assert d is None
    assert "cdcdcdcdcdcdcdcd" in why and "abababababababab" in why


def test_summary_of_this_build_is_used(tree):
    a = _args(stack="hbv_stack", steps=12, warmup=1)
    tag = bench.workload_tag(a, 524288)
    assert tag == "hbv_stack_c524288_k438_s12_w1"
    (tree / f"pmc_{tag}.json").write_text(json.dumps({"lib_sha256": "ab" * 32, "traffic_bytes_per_launch": 1.0}))
    d, why = bench.pmc_summary(a, 524288)
    assert why is None and d["traffic_bytes_per_launch"] == 1.0
    # another workload of the same build has no summary
    assert bench.pmc_summary(_args(stack="hbv_stack", steps=20, warmup=1), 524288)[0] is None


def test_committed_summaries_name_their_library():
    files = sorted((ROOT / "profiles" / "r05").glob("pmc_*.json"))
    assert files
    for f in files:
        d = json.loads(f.read_text())
        assert re.fullmatch(r"[0-9a-f]{64}", d.get("lib_sha256", "")), f.name
        assert d["workload"] in f.name and d["algorithmic_bytes_per_launch"] > 0
