"""Split a rocprofv3 kernel trace's launches of one kernel by launch shape
(grid, workgroup, LDS): the stats CSV averages every launch of a kernel name,
while gemm_x6r_kernel runs three different jobs in the C2 step (layer-0
projection, layer-0 backward pair, output-projection backward).

  python tools/x6r_launches.py <run_kernel_trace.csv> [name-substring]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "gemm_x6r_kernel"
    groups = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if pat not in r["Kernel_Name"]:
            continue
        key = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]),
               int(r["Workgroup_Size_X"]))
        groups.setdefault(key, []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print(f"{pat}: launches by grid (x, y, z) / workgroup size")
    for k, d in groups.items():
        d2 = sorted(d)
        print(f"grid {k[:3]} wg {k[3]}: {len(d)} launches, mean {sum(d) / len(d):.4f} ms, "
              f"median {d2[len(d2) // 2]:.4f} ms, min {d2[0]:.4f} ms")


if __name__ == "__main__":
    main()
