#!/usr/bin/env python3
"""Tiny beeline-style CLI: ``python tools/beeline.py -u 127.0.0.1:10000 [-e "sql"] [--nosasl]``."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(conn, sql):
    from spark_druid_olap_amd.server.hive_client import HiveError

    try:
        cur = conn.cursor().execute(sql)
        rows = cur.fetchall()
        names = [d[0] for d in cur.description or []]
        print(" | ".join(names))
        for r in rows:
            print(" | ".join("NULL" if v is None else str(v) for v in r))
        print(f"({len(rows)} rows)")
    except HiveError as e:
        print("Error:", e)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-u", default="127.0.0.1:10000")
    ap.add_argument("-e", default=None)
    ap.add_argument("-n", default="anonymous")
    ap.add_argument("--nosasl", action="store_true")
    a = ap.parse_args()
    from spark_druid_olap_amd.server.hive_client import connect

    host, port = a.u.replace("jdbc:hive2://", "").split("/")[0].split(":")
    conn = connect(host, int(port), user=a.n, sasl=not a.nosasl)
    if a.e:
        for st in a.e.split(";"):
            if st.strip():
                run(conn, st)
        return
    buf = ""
    while True:
        try:
            line = input("sdo> " if not buf else "  > ")
        except EOFError:
            break
        buf += line + "\n"
        if buf.strip().endswith(";"):
            run(conn, buf.strip().rstrip(";"))
            buf = ""
    conn.close()


if __name__ == "__main__":
    main()
