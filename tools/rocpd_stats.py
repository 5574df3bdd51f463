"""Per-kernel stats (calls, mean / total us) from a rocprofv3 SQLite output
(run_results.db, the default format when --output-format csv is not given):
  python3 tools/rocpd_stats.py gpurun_out/prof_x/run_results.db [name-substring]"""
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    q = ("select s.kernel_name, count(*), avg(d.end - d.start), sum(d.end - d.start) "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
         "group by s.kernel_name order by sum(d.end - d.start) desc")
    for name, n, avg, tot in con.execute(q):
        if flt in name:
            print(f"{n:6d} {avg / 1e3:10.2f} us {tot / 1e6:10.3f} ms  {name[:110]}")


if __name__ == "__main__":
    main()
