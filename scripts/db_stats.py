"""Per-kernel statistics from a rocprofv3 SQLite output (rocpd *_results.db): calls, total,
average, min and max duration, sorted by total time. Usage: db_stats.py <db> [top N]"""
import sqlite3
import sys


def stats(path, top=25):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), "
        "min(d.end - d.start), max(d.end - d.start) from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name "
        "order by sum(d.end - d.start) desc").fetchall()
    total = sum(r[2] for r in rows)
    out = []
    for name, n, tot, avg, mn, mx in rows[:top]:
        out.append({"kernel": name[:90], "calls": n, "total_ms": tot / 1e6, "avg_ms": avg / 1e6,
                    "min_ms": mn / 1e6, "max_ms": mx / 1e6, "pct": 100.0 * tot / total})
    return out, total / 1e6


if __name__ == "__main__":
    rows, total = stats(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
    print(f"total kernel time {total:.1f} ms")
    for r in rows:
        print(f"{r['pct']:5.1f}% {r['total_ms']:9.2f} ms {r['calls']:6d} x {r['avg_ms']:8.4f} ms  {r['kernel']}")
