"""bench.py's output contract on a real GPU, at a reduced size: one JSON line
with the metric/value/roofline keys the driver reads, the cpu_baseline leg on
rank 0, and the configs[4] end-to-end leg (pinned H2D + verify) beside the
device-resident value.  Runs bench.py as a child process (one GPU process at a
time); the full-size line is the driver's own round-end run."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(args, timeout=240):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
def test_default_line_contract_small():
    res = _run(["--blocks", "16", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0.5", "--e2e-blocks", "6"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "end_to_end"):
        assert k in res, k
    assert res["n_gpus"] == 1 and res["steps"] == 3 and res["scaling"] == "weak" and res["dtype"] == "u8"
    assert res["value"] > 0 and res["higher_is_better"] is True
    rf = res["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert rf["traffic"] is None  # PMC traffic is only quoted for the full-size launch it was measured on
    cb = res["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] == 1 and cb["kind"] in ("reference", "port")
    ac = cb["allcore"]
    assert ac["value"] > cb["value"] and ac["cores"] >= 1 and ac["kind"] == cb["kind"]
    e2e = res["end_to_end"]
    assert 0 < e2e["value"] < res["value"] and e2e["pcie_GBs"] > 0
    er = e2e["roofline"]
    assert er["bound"] == "pcie" and 0 < er["frac"] < 1.2 and er["peak"] > 10
    par = res["parity"]
    assert par["files_checked"] >= 1024 and par["mismatches"] == 0 and par["verdicts_all_ok"]


@pytest.mark.gpu
def test_zipf_and_compact_lines_carry_cpu_baseline():
    z = _run(["--workload", "zipf", "--blocks", "8", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0.3",
              "--e2e-blocks", "20"])
    assert z["roofline"]["bound"] == "hbm" and z["cpu_baseline"]["value"] > 0
    assert z["parity"]["files_checked"] > 100 and z["parity"]["mismatches"] == 0
    # configs[2] from host memory: the receive-buffer leg beside the device-resident value
    e = z["end_to_end"]
    assert 0 < e["value"] < z["value"] and e["pcie_GBs"] > 0 and e["n_buffers"] == 20 and e["inflight"] == 3
    assert e["roofline"]["bound"] == "pcie" and 0 < e["roofline"]["frac"] < 1.2
    assert e["parity"]["mismatches"] == 0 and e["parity"]["files_checked"] > 20 * 100
    assert e["per_rank"]["pcie_GBs"] and "cycled" in e["distinct_note"]
    s = _run(["--workload", "zipf_e2e", "--e2e-blocks", "8"])
    assert s["value"] > 0 and s["roofline"]["bound"] == "pcie" and s["parity"]["mismatches"] == 0
    c = _run(["--workload", "compact", "--compact-blocks", "16", "--cpu-seconds", "0.3"])
    assert c["value"] > 0 and c["cpu_baseline"]["kind"] == "port"
    assert c["unit"] == "GiB/s of live payload" and c["source_block_GiBs"] > c["value"]
    assert c["roofline"]["bound"] == "pcie" and 0 < c["roofline"]["frac"] < 1.2
    assert "256 GiB" in c["config"]["distinct_note"]  # why distinct images are cycled, beside the number
    assert c["cpu_baseline"]["allcore"]["value"] > 0 and c["cpu_baseline"]["allcore"]["cores"] >= 1


@pytest.mark.gpu
def test_ec_line_carries_cpu_baseline():
    e = _run(["--workload", "ec", "--ec-mib", "16", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0.3"])
    assert e["roofline"]["bound"] == "hbm" and e["value"] > 0
    assert e["cpu_baseline"]["value"] > 0 and e["cpu_baseline"]["kind"] in ("reference", "port")
    assert e["cpu_baseline"]["allcore"]["value"] > 0
    t = _run(["--workload", "e2e", "--compact-blocks", "8", "--cpu-seconds", "0.3"])
    assert t["roofline"]["bound"] == "pcie" and t["cpu_baseline"]["value"] > 0
    assert t["cpu_baseline"]["allcore"]["value"] > 0


@pytest.mark.gpu
def test_packet_and_compact_device_lines_carry_cpu_baseline():
    p = _run(["--workload", "packet", "--blocks", "8", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0.3"])
    assert p["cpu_baseline"]["value"] > 0 and "0x4e534654" in p["cpu_baseline"]["sample"]
    c = _run(["--workload", "compact_device", "--blocks", "8", "--steps", "2", "--warmup", "1",
              "--cpu-seconds", "0.3"])
    assert c["cpu_baseline"]["value"] > 0 and c["cpu_baseline"]["kind"] == "port"
    assert c["cpu_baseline"]["allcore"]["value"] > 0


@pytest.mark.gpu
def test_block_verify_line_carries_cpu_baseline():
    b = _run(["--workload", "block_verify", "--compact-blocks", "16", "--cpu-seconds", "0.3"])
    assert b["value"] > 0 and b["cpu_baseline"]["source_block_GiBs"] > b["cpu_baseline"]["value"] > 0
    assert b["source_block_GiBs"] > b["value"] and b["roofline"]["bound"] == "pcie"


@pytest.mark.gpu
def test_block_verify_device_and_loopback_lines():
    d = _run(["--workload", "block_verify_device", "--blocks", "8", "--steps", "2", "--warmup", "1",
              "--cpu-seconds", "0.3", "--parity-every", "4"])
    assert d["roofline"]["bound"] == "hbm" and d["value"] > 0 and d["cpu_baseline"]["value"] > 0
    assert d["parity"]["oracle_checked"] > 0
    lb = _run(["--workload", "loopback", "--steps", "1", "--cpu-seconds", "0.5"])
    assert lb["value"] > 0 and lb["roofline"]["bound"] == "pcie"
    for k in ("scalar_tfs_crc32_64KiB", "close_1_leases", "close_8_leases", "close_64_leases"):
        assert 0 < lb["latency"][k]["p50_us"] <= lb["latency"][k]["p99_us"], k
    assert lb["cpu_baseline"]["allcore"]["value"] > 0
    assert lb["resident_kernel"]["ring"] in ("device memory", "host memory")


@pytest.mark.gpu
def test_small_bodies_line():
    """Per-call latency of lone bodies: every size, the reference loop beside it, the
    crossover between them, and where the resident ring lived."""
    sb = _run(["--workload", "small_bodies", "--steps", "4"])
    assert set(sb["sizes"]) == {"32", "80", "256", "1024", "4096", "16384", "65536"}
    for k, row in sb["sizes"].items():
        assert 0 < row["scalar_us"]["p50"] <= row["scalar_us"]["p99"], k
        assert row["cpu_us"] > 0 and row["batch_us_per_frame"]["p50"] > 0, k
    assert sb["higher_is_better"] is False and sb["cpu_kind"] in ("reference", "port")
    assert 80 < sb["crossover_bytes"] < 65536
    assert sb["resident_ring"] in ("device memory", "host memory")


@pytest.mark.gpu
def test_compact_files_line():
    c = _run(["--workload", "compact_files", "--file-blocks", "2", "--cpu-seconds", "0.5"])
    assert c["value"] > 0 and c["source_block_GiBs"] > c["value"]
    assert c["roofline"]["bound"] == "host-io" and 0 < c["roofline"]["frac"]
    assert c["cpu_baseline"]["value"] > 0 and c["cpu_baseline"]["kind"] == "port"
