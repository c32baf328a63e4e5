"""CPU checks of the measurement tooling: tools/pmc_summary.py folds rocprofv3
counter passes with the gfx950 FETCH_SIZE x2 correction (MI355X_MICROARCH.md §HBM)."""
import json
import os
import subprocess
import sys

from conftest import ROOT

KERNEL = "void tfscrc::crc_files_kernel<1, 4, 3>(unsigned char const*)"
HDR = ('"Correlation_Id","Dispatch_Id","Agent_Id","Queue_Id","Process_Id","Thread_Id","Grid_Size","Kernel_Id",'
       '"Kernel_Name","Workgroup_Size","LDS_Block_Size","Scratch_Size","VGPR_Count","Accum_VGPR_Count","SGPR_Count",'
       '"Counter_Name","Counter_Value","Start_Timestamp","End_Timestamp"')


def _pass(path, counter, values):
    with open(path, "w") as fh:
        fh.write(HDR + "\n")
        for i, v in enumerate(values):
            fh.write('%d,%d,"Agent 2",1,1,1,262144,13,"%s",1024,159744,0,52,0,112,"%s",%f,0,1\n'
                     % (i, i, KERNEL, counter, v))
        fh.write('99,99,"Agent 2",1,1,1,256,3,"tfscrc::synth_fill_kernel()",256,0,0,8,0,16,"%s",1.0,0,1\n' % counter)


def test_pmc_summary_corrections(tmp_path):
    _pass(tmp_path / "f.csv", "FETCH_SIZE", [1000.0, 1002.0, 1001.0])
    _pass(tmp_path / "w.csv", "WRITE_SIZE", [10.0, 10.0, 12.0])
    _pass(tmp_path / "r.csv", "TCC_EA0_RDREQ_sum", [16016.0] * 3)
    stats = tmp_path / "ks.csv"
    stats.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
                     '"%s",3,3000,1000.0,90.0,990,1010,5.0\n' % KERNEL)
    out = tmp_path / "p" / "s.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), "--tag", "t", "--stats",
                        str(stats), "--out", str(out), "--algo-bytes", "2048000", str(tmp_path / "f.csv"),
                        str(tmp_path / "w.csv"), str(tmp_path / "r.csv")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    d = json.loads(out.read_text())
    assert d["read_bytes_corrected"] == 1001.0 * 1024 * 2          # median FETCH_SIZE (KiB) x 2
    assert d["write_bytes"] == 10.0 * 1024
    assert d["read_bytes_from_rdreq_x128"] == 16016.0 * 128
    assert d["rocprof_kernel_stats"]["avg_ns"] == 1000.0
    assert abs(d["traffic_over_algorithmic"] - (1001.0 * 2048 + 10240) / 2048000) < 1e-12
