"""CPU: bench.py pairs PMC counters with a launch only when they were measured on the same
library: profiles/pmc_traffic.json and pmc_valu.json entries carry the sha256
prefix of libviterbi_amd.so, and any other binary's counters read as null."""
import hashlib
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

KEY = "K7_soft_F4096_L1024"


@pytest.fixture
def fake_repo(tmp_path, monkeypatch):
    lib = tmp_path / "convolutionalencdec_amd" / "lib"
    lib.mkdir(parents=True)
    (lib / "libviterbi_amd.so").write_bytes(b"not a real library")
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    return tmp_path, hashlib.sha256(b"not a real library").hexdigest()[:16]


def write(root, name, data):
    (root / "profiles" / name).write_text(data if isinstance(data, str) else json.dumps(data))


def test_matching_stamp_is_used(fake_repo):
    root, sha = fake_repo
    assert bench.lib_sha16() == sha
    write(root, "pmc_traffic.json", {KEY: {"bytes_per_launch": 9476511, "lib_sha16": sha}})
    write(root, "pmc_valu.json", {KEY: {"valu_wave_insts_per_launch": 11270238, "waves_per_launch": 2048, "lib_sha16": sha}})
    assert bench.load_traffic(KEY) == 9476511
    assert bench.load_valu(KEY)["valu_wave_insts_per_launch"] == 11270238


def test_other_library_reads_null(fake_repo):
    root, sha = fake_repo
    write(root, "pmc_traffic.json", {KEY: {"bytes_per_launch": 9476511, "lib_sha16": "0" * 16}})
    write(root, "pmc_valu.json", {KEY: {"valu_wave_insts_per_launch": 1, "lib_sha16": sha[::-1]}})
    assert bench.load_traffic(KEY) is None
    assert bench.load_valu(KEY) is None


@pytest.mark.parametrize("content", [None, "{not json", json.dumps({"other": {"bytes_per_launch": 1}}),
                                     json.dumps({KEY: 5}), json.dumps({KEY: {"bytes_per_launch": 1}})])
def test_missing_or_malformed_reads_null(fake_repo, content):
    root, _ = fake_repo
    if content is not None:
        write(root, "pmc_traffic.json", content)
    assert bench.load_traffic(KEY) is None


def test_committed_counter_files_are_stamped():
    """Every committed entry names the library it was measured on (a 16-hex-digit stamp)."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for name in ("pmc_traffic.json", "pmc_valu.json"):
        with open(os.path.join(repo, "profiles", name)) as fh:
            data = json.load(fh)
        assert data
        for key, ent in data.items():
            assert len(ent["lib_sha16"]) == 16 and int(ent["lib_sha16"], 16) >= 0, (name, key)
