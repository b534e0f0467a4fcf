"""Top kernels of a ``rocprofv3 --kernel-trace --stats`` output directory, as a text table.

  python scripts/prof_summary.py gpurun_out/prof_topk [N]
"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    files = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)
    if not files:
        raise SystemExit(f"no kernel_stats.csv under {d}")
    rows = list(csv.DictReader(open(files[0])))
    for r in rows[:top]:
        print(f"{r['Name'][:100]:100s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:10.2f}us "
              f"{float(r['Percentage']):6.2f}%")


if __name__ == "__main__":
    main()
