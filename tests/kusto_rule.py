"""kusto_ingest.py's file selection and PerfLogsMPI row schema, restated for
the tests (the script itself needs azure + a network Kusto endpoint and is not
importable here).

select(): /root/reference/kusto_ingest.py:32-40 — regular files in the ingest
directory whose name starts with "tcp" (case-insensitive), sorted by mtime,
all but the newest n (the reference passes n = -f, the flow count).

parse_row(): one CSV line of the schema the reference writes
(mpi_perf.c:550-554): Timestamp:datetime, JobId:string, Rank:int,
VMCount:int, LocalIP:string, RemoteIP:string, NumOfFlows:int,
BufferSize:int, NumOfBuffers:int, TimeTakenms:real, RunId:int.
"""
from __future__ import annotations

import datetime
import ipaddress
import os


def select(kusto_dir: str, n: int) -> list[str]:
    files = [os.path.join(kusto_dir, f) for f in os.listdir(kusto_dir)
             if os.path.isfile(os.path.join(kusto_dir, f)) and f.lower().startswith("tcp")]
    files.sort(key=os.path.getmtime)
    return files[:-n]


COLUMNS = ["Timestamp", "JobId", "Rank", "VMCount", "LocalIP", "RemoteIP", "NumOfFlows", "BufferSize",
           "NumOfBuffers", "TimeTakenms", "RunId"]


def parse_row(line: str) -> dict:
    f = line.rstrip("\n").split(",")
    if len(f) != len(COLUMNS):
        raise ValueError(f"{len(f)} fields, want {len(COLUMNS)}: {line!r}")
    row = dict(zip(COLUMNS, f))
    row["Timestamp"] = datetime.datetime.strptime(f[0], "%Y-%m-%d %H:%M:%S")
    for k in ("Rank", "VMCount", "NumOfFlows", "BufferSize", "NumOfBuffers", "RunId"):
        row[k] = int(row[k])
    row["TimeTakenms"] = float(row["TimeTakenms"])
    for k in ("LocalIP", "RemoteIP"):
        row[k] = str(ipaddress.IPv4Address(row[k]))   # plain IPv4, as the reference writes
    return row
