"""Print one training step's kernel timeline from a rocprofv3 results DB (tools/timeline.py DB [marker])."""
import sqlite3
import sys

db = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "photo_loss_fwd"
which = int(sys.argv[3]) if len(sys.argv) > 3 else -3  # occurrence index of the marker
c = sqlite3.connect(db)
rows = list(c.execute("select name,start,end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if marker in r[0]]
print("marker occurrences:", len(idx))
i0, i1 = idx[which], idx[which + 1]
t0 = rows[i0][1]
busy = 0
for r in rows[i0:i1]:
    busy += r[2] - r[1]
    print(f"{(r[1] - t0) / 1e3:9.1f} {(r[2] - r[1]) / 1e3:8.1f}  {r[0][:100]}")
span = rows[i1][1] - t0
print(f"step span {span / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us, kernels {i1 - i0}")
