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


def test_kernel_time_stamp(fake_repo):
    """roofline.rocprof_avg_ms comes from profiles/kernel_time.json only for this library."""
    root, sha = fake_repo
    write(root, "kernel_time.json", {KEY: {"avg_ns": 32473.3, "kernel": "k7_lds_kernel<...>", "calls": 57,
                                           "lib_sha16": sha}})
    assert bench.load_kernel_time(KEY)["avg_ns"] == 32473.3
    write(root, "kernel_time.json", {KEY: {"avg_ns": 32473.3, "lib_sha16": "f" * 16}})
    assert bench.load_kernel_time(KEY) is None
    write(root, "kernel_time.json", {KEY: {"avg_ns": "x", "lib_sha16": sha}})
    assert bench.load_kernel_time(KEY) is None


def _block(**kw):
    args = dict(alg_bytes=8962048, avg_ms=0.0316, n_avg=50, kern_ms=0.0326, launch_ms=[0.034, 0.0339, 0.0391],
                issue_us=4.4, state_steps=4096 * 64 * 1030, kernel="k7_lds")
    args.update(kw)
    return bench.roofline_block(**args)


def test_roofline_fields_named_for_what_they_time():
    """kernel_avg_ms (back-to-back launches) drives achieved / frac; the timed region's span is
    timed_span_ms (verdict r03 item 5); the host's issue time sits beside it and flags a
    kernel_avg_ms that issue could explain."""
    r = _block()
    assert r["kernel_avg_ms"] == 0.0316 and r["timed_span_ms"] == 0.0326
    assert r["achieved"] == pytest.approx(8962048 / 31.6e-6 / 1e9, rel=1e-4)
    assert r["frac"] == pytest.approx(r["achieved"] / 8000.0, rel=1e-4)
    assert r["host_issue_us_per_launch"] == 4.4 and r["kernel_avg_issue_bound"] is False
    assert _block(issue_us=30.0)["kernel_avg_issue_bound"] is True
    assert r["per_launch_pass_ms"]["max"] == 0.0391 and r["traffic"] is None and r["rocprof_avg_ms"] is None
    assert _block(kernel_time={"avg_ns": 32030.0})["rocprof_avg_ms"] == 0.03203


def test_valu_secondary_against_two_cycle_peak():
    """roofline.secondary: the 2-cycle wave64 peak (1,228.8 G/s, MI355X_MICROARCH.md) is `peak`,
    the 4-cycle rate a named field beside it, and the kernel's issue-priced mix (tools/isa_mix.py)
    its own bound (verdict r04 item 5)."""
    mix = {"priced_peak_G": 607.9, "valu_per_wave_step": 5.0, "priced_cycles_per_wave_step": 20.212}
    r = _block(valu={"valu_wave_insts_per_launch": 11270238}, mix=mix)["secondary"]
    ach = 11270238 / 31.6e-6 / 1e9
    assert r["achieved"] == pytest.approx(ach, abs=0.01)
    assert r["peak"] == 1228.8 and r["frac"] == pytest.approx(ach / 1228.8, abs=1e-4)
    assert r["peak_4cycle"] == 614.4 and r["frac_4cycle"] == pytest.approx(ach / 614.4, abs=1e-4)
    assert r["issue_priced"]["peak"] == 607.9 and r["issue_priced"]["frac"] == pytest.approx(ach / 607.9, abs=1e-4)
    assert r["state_steps_per_s"] == round(4096 * 64 * 1030 / 31.6e-6)
    no = _block()["secondary"]
    assert "frac" not in no and "issue_priced" not in no


@pytest.mark.parametrize("kernel", ["k7_lds", "k7_lds_loop", "k7_split_loop", "k9", "lds_path"])
def test_secondary_note_per_kernel(kernel):
    r = _block(kernel=kernel)["secondary"]
    assert r["kernel"] == kernel and r["note"].startswith(bench.KERNEL_NOTES[kernel])
    assert len({bench.KERNEL_NOTES[k] for k in bench.KERNEL_NOTES}) == len(bench.KERNEL_NOTES)


def test_isa_mix_stamp(fake_repo):
    root, sha = fake_repo
    write(root, "isa_mix.json", {"k7_lds/soft": {"priced_peak_G": 607.9, "lib_sha16": sha},
                                 "k9/hard": {"priced_peak_G": 606.5, "lib_sha16": "0" * 16}})
    assert bench.load_isa_mix("k7_lds", True)["priced_peak_G"] == 607.9
    assert bench.load_isa_mix("k7_lds", False) is None
    assert bench.load_isa_mix("k9", False) is None


def test_committed_isa_mix_covers_the_bench_configs():
    """profiles/isa_mix.json (tools/isa_mix.py) prices the kernels of every BASELINE config line
    from the 48-step chunk loop: 48 v_pk_min per metric register."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(repo, "profiles", "isa_mix.json")) as fh:
        mix = json.load(fh)
    for key, regs in (("k7_lds/soft", 1), ("k7_lds/hard", 1), ("k7_split_loop/soft", 1), ("k7_split_loop/hard", 1),
                      ("k7_lds_loop/soft", 1), ("k9/hard", 4)):
        ent = mix[key]
        assert ent["mix"]["pk_min"] == 48 * regs and ent["loop_steps"] == 48, key
        assert 500 < ent["priced_peak_G"] < 1228.8, key
        assert len(ent["lib_sha16"]) == 16


# ---- tools/kernel_time_summary.py: the timed window and the stamp's source ----

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import kernel_time_summary as kts  # noqa: E402


def _spans(bursts):
    """[(start, end)] of back-to-back 32-us dispatches in bursts separated by the given gaps."""
    out, t = [], 0
    for n, gap in bursts:
        t += gap
        for _ in range(n):
            out.append((t, t + 32_000))
            t += 32_000 + 500
    return out


def test_timed_window_skips_the_isolated_first_dispatch():
    # bench.py: one isolated dispatch, the 5-launch warm-up burst, the 20 timed launches, the
    # 51-launch average pass, the per-launch pass (events open ~5 us gaps)
    sp = _spans([(1, 0), (5, 400_000), (20, 70_000), (51, 45_000)] + [(1, 6_000)] * 20)
    assert kts.timed_window(sp, 5, 20) == 6
    assert kts.timed_window(_spans([(5, 0), (20, 70_000)]), 5, 20) == 5


@pytest.mark.parametrize("trace", ["profiles/r04/final/kernel_trace_bench_driver_cmd.csv",
                                   "profiles/r05/final/kernel_trace_bench_driver_cmd.csv"])
def test_timed_window_on_committed_traces(trace):
    import csv

    rows = [r for r in csv.DictReader(open(os.path.join(REPO, trace))) if "k7_lds_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    lo = kts.timed_window(sp, 5, 20)
    assert lo == 6  # the driver's command: dispatch 0 alone, 1-5 the warm-up, 6-25 timed
    assert all(sp[i][0] - sp[i - 1][1] < 10_000 for i in range(lo + 1, lo + 20))
    assert sp[lo][0] - sp[lo - 1][1] > 10_000


def test_summary_refuses_unstamped_or_ambiguous_runs(tmp_path):
    import subprocess

    script = os.path.join(REPO, "tools", "kernel_time_summary.py")
    (tmp_path / "a").mkdir()
    (tmp_path / "a" / "run_kernel_stats.csv").write_text("Name,Calls,AverageNs\n")
    r = subprocess.run([sys.executable, script, str(tmp_path), "K"], capture_output=True, text=True)
    assert r.returncode != 0 and "lib_sha16.txt" in (r.stderr + r.stdout)
    (tmp_path / "b").mkdir()
    (tmp_path / "b" / "run_kernel_stats.csv").write_text("Name,Calls,AverageNs\n")
    r = subprocess.run([sys.executable, script, str(tmp_path), "K"], capture_output=True, text=True)
    assert r.returncode != 0 and "exactly one run" in (r.stderr + r.stdout)
