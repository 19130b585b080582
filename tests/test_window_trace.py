"""tools/window_trace.py groups a kernel trace of bench.py's deletion window (CPU, synthetic trace).

The dispatch order it assumes is bench.deletion_window's: run-up to the hand-off, `warm` more steps,
then per mode `warm` untimed steps from the hand-off and the timed window, then the checked
reference-order run. Each synthetic element dispatch lasts a duration that encodes its group, so a
wrong split shows up as a wrong mean."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(tmp_path, groups):
    rows, t = [], 0
    for dur_ns, n in groups:
        for _ in range(n):
            for name, d in (("void hk::k_nodal<3, false, false>(hk::NodalArgs)", 50_000),
                            ("void hk::k_bc(hk::BCArgs)", 7_000),
                            ("void hk::k_element_pipe<true, false, true, true, 3, false, 2>(hk::ElemArgs)", dur_ns)):
                rows.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + d})
                t += d + 1000
    d = tmp_path / "kt"
    d.mkdir()
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)
    return d


def test_window_trace_groups_the_bench_protocol(tmp_path):
    n, warm = 20, 100
    # run-up (to the hand-off, then the continuation), headline warm + window, other warm + window, check
    kt = _trace(tmp_path, [(800_000, 300), (810_000, warm), (900_000, warm), (820_000, n), (950_000, warm),
                           (990_000, n), (1_100_000, n)])
    line = {"config": {"element_mode": "fused",
                       "deletion_window": {"first_step": 7941, "steps": n, "warm_steps_per_mode": warm}}}
    log = tmp_path / "bench.log"
    log.write_text("noise\n" + json.dumps(line) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "window_trace.py"), "--kt", str(kt),
                          "--log", str(log)], check=True, capture_output=True, text=True).stdout
    d = json.loads(out)
    assert d["run_up"]["element_mean_ms"] == 0.81 and d["run_up"]["steps"] == [7921, 7940]
    assert d["fused"]["element_mean_ms"] == 0.82 and d["fused"]["steps"] == [7941, 7960]
    assert d["exact"]["element_mean_ms"] == 0.99
    assert d["checked_run_after_upload"]["element_mean_ms"] == 1.1
    assert d["fused"]["nodal_bc_mean_ms"] == 0.057


def test_window_trace_groups_the_control_protocol(tmp_path):
    n = 20
    # tools/window_control.py: run-up, then per mode one planning step and the window
    kt = _trace(tmp_path, [(800_000, 440), (700_000, 1), (830_000, n), (700_000, 1), (960_000, n)])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "window_trace.py"), "--kt", str(kt),
                          "--first", "441"], check=True, capture_output=True, text=True).stdout
    d = json.loads(out)
    assert d["run_up"]["element_mean_ms"] == 0.8 and d["run_up"]["steps"] == [421, 440]
    assert d["fused"]["element_mean_ms"] == 0.83
    assert d["exact"]["element_mean_ms"] == 0.96
