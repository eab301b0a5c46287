set -o pipefail
# k-means kernel profile (summaries written on the box)
O=$GRAFT_REPO_ROOT/gpurun_out/r3s2km
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_km -o km -- python3 $GRAFT_REPO_ROOT/bench/kmeans_bench.py > $O/prof_km.log 2>&1 && \
python3 $GRAFT_REPO_ROOT/bench/summarize_db.py /tmp/prof_km/km_results.db 40 > $O/stats.md && \
python3 - <<'PY' > $O/timeline.txt
import sqlite3
c = sqlite3.connect("/tmp/prof_km/km_results.db")
rows = c.execute("select name, start, end from kernels order by start").fetchall()
t0 = rows[-60][1]
for n, s, e in rows[-60:]:
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  {n[:90]}")
PY
