"""Copies the rocprofv3 summaries of a GPU session into profiles/ (tracked)
and derives profiles/pmc_latest.json (HBM bytes per launch) for bench.py.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads and
WRITE_SIZE is exact for 16 B/lane stores (MI355X_MICROARCH.md, HBM)."""
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = ROOT / "gpurun_out" / "prof"
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)
shutil.copy(src / "trace" / "run_kernel_stats.csv", dst / f"{tag}_bench_kernel_stats.csv")
shutil.copy(src / "pmc_summary.txt", dst / f"{tag}_pmc_summary.txt")
pmc = json.loads((src / "pmc_summary.json").read_text())
sys.path.insert(0, str(ROOT))
from bench import kernel_source_sha256  # noqa: E402

latest = {"source": f"profiles/{tag}_pmc_summary.txt", "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024",
          # the HIP sources the counters were taken of: bench.py reports `traffic` only while they match
          "kernel_source_sha256": kernel_source_sha256()}
for k, v in pmc.items():
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        latest[k] = {"hbm_bytes_per_launch": int((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024),
                     "fetch_kb": v["FETCH_SIZE"], "write_kb": v["WRITE_SIZE"]}
        if "GRBM_GUI_ACTIVE" in v:
            # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles: per XCD it is the launch's length in
            # GPU clock cycles, independent of the clock the chip ran at
            latest[k]["grbm_gui_active"] = v["GRBM_GUI_ACTIVE"]
            latest[k]["cycles_per_launch"] = int(v["GRBM_GUI_ACTIVE"] / 8)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT"):
            if c in v:
                latest[k][c] = v[c]
(dst / "pmc_latest.json").write_text(json.dumps(latest, indent=1) + "\n")
print(json.dumps(latest, indent=1))
