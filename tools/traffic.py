"""Per-launch HBM traffic of the round kernel from rocprofv3 PMC passes
(experiment tool; writes the summary bench.py reports as roofline.traffic).

    python tools/traffic.py <fetch_dir> <write_dir> <kernel_substring> <workload_key> [--last N]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (summed over the XCDs' TCC
channels).  Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM
section): on gfx950 FETCH_SIZE reports half of the bytes of wide coalesced
streaming reads, so the streaming-read part is doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Our reads are mostly such streams plus 16-B
gathers, so the whole FETCH_SIZE is doubled (an upper estimate for the gather
part, stated in DESIGN.md).  Infinity-Cache hits are counted, not excluded.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402


def main():
    fdir, wdir, sub, key = sys.argv[1:5]
    last = 10
    for a in sys.argv[5:]:
        if a.startswith("--last="):
            last = int(a.split("=")[1])
    f = summarise(fdir, sub, last=last)
    w = summarise(wdir, sub, last=last)
    fetch_kib, write_kib = f["FETCH_SIZE"], w["WRITE_SIZE"]
    rec = {
        "kernel_substring": sub,
        "dispatches_averaged": min(f["_dispatches"], w["_dispatches"]),
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib_raw": write_kib,
        "fetch_correction": 2.0,
        "hbm_bytes_per_launch": (2.0 * fetch_kib + write_kib) * 1024.0,
    }
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    d = {}
    if os.path.exists(path):
        with open(path) as fh:
            d = json.load(fh)
    d[key] = rec
    with open(path, "w") as fh:
        json.dump(d, fh, indent=1, sort_keys=True)
    print(json.dumps({key: rec}, indent=1))


if __name__ == "__main__":
    main()
