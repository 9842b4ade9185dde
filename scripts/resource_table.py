"""Per-kernel registers / scratch / occupancy of the library's kernels (hipcc remarks).

  python3 scripts/resource_table.py [--scratch-only] [file.hip ...]
"""
import re
import subprocess
import sys

SRC = "round_amd/csrc"
FILES = ["psg_otr.hip", "psg_lv.hip", "psg_floodmin.hip", "psg_kset.hip", "psg_benor.hip", "psg_slv.hip",
         "psg_kset_es.hip", "psg_epsilon.hip", "psg_schedule.hip"]
FIELDS = {"TotalSGPRs": "sgpr", "VGPRs": "vgpr", "ScratchSize [bytes/lane]": "scratch",
          "Occupancy [waves/SIMD]": "waves", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill"}


def table(files):
    rows = []
    for f in files:
        out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c", f,
                              "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"], cwd=SRC,
                             capture_output=True, text=True).stderr
        cur = None
        for line in out.splitlines():
            m = re.search(r"remark: \s*(.+?): (.+?) \[-Rpass", line)
            if not m:
                continue
            k, v = m.group(1).strip(), m.group(2).strip()
            if k == "Function Name":
                cur = {"kernel": v}
                rows.append(cur)
            elif cur is not None and k in FIELDS:
                cur[FIELDS[k]] = int(v)
    return rows


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    only = "--scratch-only" in sys.argv
    for r in table(args or FILES):
        if "_kernel" not in r["kernel"] or (only and not r.get("scratch")):
            continue
        print(f"{r['kernel'][:70]:70s} sgpr {r.get('sgpr')} vgpr {r.get('vgpr')} scratch {r.get('scratch')} "
              f"waves {r.get('waves')} spill s{r.get('sgpr_spill')}/v{r.get('vgpr_spill')}")
