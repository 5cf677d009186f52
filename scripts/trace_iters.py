"""k_corr / k_solve duration of every iteration of the last align() in a rocprofv3 kernel trace."""
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
corr = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_corr" in r["Kernel_Name"]][-n:]
solve = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_solve" in r["Kernel_Name"]][-n:]
print("k_corr us per iteration:", " ".join(f"{x:.0f}" for x in corr))
print("k_solve us per iteration:", " ".join(f"{x:.0f}" for x in solve))
print(f"sum k_corr {sum(corr):.0f} us, mean {sum(corr)/len(corr):.1f}; sum k_solve {sum(solve):.0f} us")
