#!/usr/bin/env python3
"""Regenerate tests/golden/geometry.json from the reference itself.

Run in the build container (needs /root/reference):  python tests/golden/make_geometry_golden.py

oracle/_ref/ref_geometry is recode.cpp:233-471 (r_scan8, scan_8, reverse_scan_8, the zigzag
tables, test_reverse_scan8, get_neighbor_sub_mb) compiled from the reference's own source by
`make -C oracle ref` (oracle/ref_geometry_driver.cpp).  Its output is data only: the tables and
get_neighbor_sub_mb's result for above in {0,1}, sub_mb_size in {4,8,15,16,64}, scan8_index 0..50,
mb_x, mb_y in {0,1} -- the reference's answer for every neighbour the model can ask for
(SURVEY.md §8a row a17).
"""
import json
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]


def main():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "ref"], check=True)
    out = subprocess.run([str(ROOT / "oracle" / "_ref" / "ref_geometry")], check=True, capture_output=True,
                         text=True).stdout
    data = json.loads(out)
    data["_source"] = ("oracle/_ref/ref_geometry: /root/reference/recode.cpp:233-471 compiled as-is "
                       "(oracle/Makefile target ref); columns of neighbors: above, sub_mb_size, scan8_index, "
                       "mb_x, mb_y, returned, out.mb_x, out.mb_y, out.scan8_index")
    path = ROOT / "tests" / "golden" / "geometry.json"
    with open(path, "w") as f:
        f.write("{\n")
        keys = [k for k in data if k != "neighbors"]
        for k in keys:
            f.write(f" {json.dumps(k)}: {json.dumps(data[k])},\n")
        f.write(' "neighbors": [\n')
        f.write(",\n".join("  " + json.dumps(r) for r in data["neighbors"]))
        f.write("\n ]\n}\n")
    print(f"wrote {path} ({len(data['neighbors'])} neighbour cases)")


if __name__ == "__main__":
    main()
