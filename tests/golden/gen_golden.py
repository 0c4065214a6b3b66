#!/usr/bin/env python3
"""Generate tests/golden/ref_runs.json by running the COMPILED REFERENCE.

Runs /root/reference/mpi_perf.c, compiled by `make -C oracle ref` with the
image's MPICH 3.3.2 (no stand-ins), under MPICH's mpiexec with the PMPI
interposer oracle/ref_shim.c (fake two hosts + receive accounting), over a
matrix of modes / PPN / sizes / iteration counts and the reference's error
cases.  Everything variable (UUIDs, timestamps, times) is
masked; what remains is the reference's observable contract:

  * exit status, stderr INFO lines (group / group_size / group_rank / peer),
  * the CSV records (field by field; time kept as a number only for format),
  * the log-file name shape,
  * per-rank receive accounting: receives completed, bytes, and the sum of
    oracle_checksum() of each received payload.

Only runnable where /root/reference exists (this container).  The output is
committed; tests read only the JSON.
"""
from __future__ import annotations

import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ORACLE = os.path.join(REPO, "oracle")
REF_BIN = os.path.join(ORACLE, "_ref", "mpi_perf")
WRAP = os.path.join(ORACLE, "ref_wrap.sh")
MPIEXEC = "/opt/conda/bin/mpiexec"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_runs.json")

UUID_RE = re.compile(r"[0-9a-f]{8}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{12}")
INFO_RE = re.compile(
    r"INFO: (\S+), rank (\d+) out of (\d+) ranks, my_group: (\d+), group_size: (\d+), group_rank: (\d+), "
    r"my_peer: (-?\d+), hostname: (\S+) \((\S*)\), peer_host: (\S+) \((\S*)\)")
SUMMARY_RE = re.compile(r"\[Run#: (\d+)\]: Total time: [0-9.]+ ms, Min: [0-9.]+ ms, Max: [0-9.]+ ms, Avg: [0-9.]+ ms")
LOGNAME_RE = re.compile(r"^tcp-([0-9a-f-]{36})-(\d+)-(\d{4}-\d\d-\d\d-\d\d-\d\d-\d\d)\.log$")


def run_case(name, np_, ppn, args, group1_lines=("vm",), host1="vm", host0="runsc", timeout=120):
    tmp = tempfile.mkdtemp(prefix="ref_")
    try:
        g1 = os.path.join(tmp, "group1")
        with open(g1, "w") as f:
            f.write("".join(line + "\n" for line in group1_lines))
        logs = os.path.join(tmp, "logs")
        os.mkdir(logs)
        argv = [a.replace("@G1", g1).replace("@LOGS", logs) for a in args]
        env = dict(os.environ, PPN=str(ppn), HOST1=host1, HOST0=host0, SHIM_OUT=os.path.join(tmp, "shim"))
        cmd = [MPIEXEC, "-np", str(np_), "-genv", "PPN", str(ppn), "-genv", "HOST1", host1, "-genv", "HOST0", host0,
               "-genv", "SHIM_OUT", os.path.join(tmp, "shim"), WRAP, REF_BIN] + argv
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=tmp)
        err = p.stderr
        info = []
        for m in INFO_RE.finditer(err):
            info.append(dict(name=m[1], rank=int(m[2]), world=int(m[3]), group=int(m[4]), group_size=int(m[5]),
                             group_rank=int(m[6]), peer=int(m[7]), host=m[8], ip=m[9], peer_host=m[10],
                             peer_ip=m[11]))
        info.sort(key=lambda d: d["rank"])
        summaries = sorted(int(m[1]) for m in SUMMARY_RE.finditer(err))
        files, records = [], []
        for path in sorted(glob.glob(os.path.join(logs, "*"))):
            base = os.path.basename(path)
            m = LOGNAME_RE.match(base)
            files.append(dict(shape_ok=bool(m), rank=int(m[2]) if m else None))
            with open(path) as f:
                for line in f:
                    fld = line.rstrip("\n").split(",")
                    records.append(dict(
                        n_fields=len(fld),
                        timestamp_ok=bool(re.match(r"^\d{4}-\d\d-\d\d \d\d:\d\d:\d\d$", fld[0])),
                        uuid_ok=bool(UUID_RE.fullmatch(fld[1])),
                        rank=int(fld[2]), vmcount=int(fld[3]), local_ip=fld[4], remote_ip=fld[5],
                        flows=int(fld[6]), buffer_size=int(fld[7]), num_buffers=int(fld[8]),
                        time_ms_text=fld[9], run_id=int(fld[10]), line_masked=",".join(["T", "U"] + fld[2:9] + ["X"] + fld[10:])))
        records.sort(key=lambda r: (r["rank"], r["run_id"]))
        n_records = len(records)
        records = records[:8]
        shim = {}
        for path in glob.glob(os.path.join(tmp, "shim.*.json")):
            d = json.load(open(path))
            shim[str(d["rank"])] = {k: d[k] for k in ("recv_done", "recv_bytes", "recv_digest", "waitall_calls",
                                                      "waitall_reqs")}
        dotnet = sorted(re.findall(r"^dotnet .*$", err, flags=re.M))
        messages = []
        for key in ("invalid group_size", "getaddrinfo error", "Usage: <program>", "cannot open group1 file",
                    "failed to read OMPI_COMM_WORLD_LOCAL_RANK"):
            if key in err:
                messages.append(key)
        return dict(name=name, np=np_, ppn=ppn, args=args, group1_lines=list(group1_lines), host1=host1, host0=host0,
                    returncode=p.returncode, uuid_printed=bool(re.search(r"UUID: " + UUID_RE.pattern, err)),
                    info=info, summaries=summaries, files=files, records=records, n_records=n_records, shim=shim, messages=messages, dotnet=dotnet)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    if not os.path.exists(REF_BIN):
        sys.exit("build the reference first: make -C oracle ref")
    cases = []
    # --- loop modes x PPN x sizes (parity of pairing, records, payloads) ---
    for mode, flag in (("pingpong", []), ("nonblocking", ["-x", "1"]), ("unidir", ["-u", "1"])):
        for ppn in (1, 2, 4):
            for B, iters in ((1, 10), (8, 10), (4096, 7), (456131, 3)):
                cases.append(run_case(f"{mode}_p{ppn}_b{B}_i{iters}", 2 * ppn, ppn,
                                      ["-f", "@G1", "-n", "1", "-p", str(ppn), "-r", "3", "-i", str(iters),
                                       "-b", str(B), "-l", "@LOGS"] + flag))
    # --- nonblocking window quirk: slot 255 of each window is never waited ---
    for iters in (255, 256, 257, 512, 600):
        cases.append(run_case(f"nonblocking_window_i{iters}", 2, 1,
                              ["-f", "@G1", "-n", "1", "-p", "1", "-r", "2", "-i", str(iters), "-b", "64", "-l",
                               "@LOGS", "-x", "1"]))
    # --- default buffer size / iterations (mpi_perf.c:14-15, :388-392) ---
    cases.append(run_case("defaults_unidir", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-u", "1", "-r", "2",
                                                    "-l", "@LOGS"]))
    cases.append(run_case("zero_bytes_pingpong", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-r", "2", "-i", "5",
                                                        "-b", "0", "-l", "@LOGS"]))
    # the ack is tx[0:1) even at -b 0 (mpi_perf.c:142): a byte of a 0-byte block
    cases.append(run_case("zero_bytes_unidir", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-r", "2", "-i", "5",
                                                      "-b", "0", "-l", "@LOGS", "-u", "1"]))
    cases.append(run_case("zero_bytes_nonblocking", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-r", "2", "-i", "5",
                                                           "-b", "0", "-l", "@LOGS", "-x", "1"]))
    # --- group rule: case-insensitive prefix over the processor name ---
    cases.append(run_case("group_upper_prefix_line", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-r", "2", "-i", "3",
                                                            "-b", "8", "-l", "@LOGS"], group1_lines=("VMX",)))
    cases.append(run_case("group_two_lines", 4, 2, ["-f", "@G1", "-n", "2", "-p", "2", "-u", "1", "-r", "2", "-i",
                                                    "3", "-b", "8", "-l", "@LOGS"], group1_lines=("nohost", "vm")))
    # --- run 0 is the warm-up: -r 1 writes no record (mpi_perf.c:545) ---
    cases.append(run_case("one_run_no_records", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-r", "1", "-i", "3",
                                                       "-b", "8", "-l", "@LOGS"]))
    # --- summary printed by rank 0 every 1000 runs (mpi_perf.c:564) ---
    cases.append(run_case("summary_every_1000", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-r", "1002", "-i", "1",
                                                       "-b", "1", "-l", "@LOGS"]))
    # --- flag interplay and degenerate loops ---
    cases.append(run_case("unidir_wins_over_nonblocking", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-u", "1", "-x",
                                                                 "1", "-r", "2", "-i", "4", "-b", "16", "-l", "@LOGS"]))
    cases.append(run_case("zero_runs", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-r", "0", "-i", "4", "-b", "16",
                                              "-l", "@LOGS"]))
    cases.append(run_case("zero_iters", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-r", "3", "-i", "0", "-b", "16",
                                               "-l", "@LOGS"]))
    # --- the .NET launcher mode only prints its command lines (mpi_perf.c:147-168) ---
    cases.append(run_case("dotnet_print_only", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-d", "1", "-r", "2", "-i",
                                                      "7", "-b", "64", "-l", "@LOGS"]))
    # --- error exits ---
    cases.append(run_case("err_bidir_no_ppn_sigfpe", 2, 1, ["-f", "@G1", "-n", "1", "-r", "2", "-i", "3", "-b", "8",
                                                           "-l", "@LOGS"]))
    cases.append(run_case("err_unidir_no_ppn_sigfpe", 2, 1, ["-f", "@G1", "-n", "1", "-u", "1", "-r", "2", "-i",
                                                            "3", "-b", "8", "-l", "@LOGS"]))
    cases.append(run_case("err_unknown_flag", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-z", "1"]))
    cases.append(run_case("err_h_flag", 2, 1, ["-h", "1"]))
    cases.append(run_case("err_bad_group_size", 2, 1, ["-f", "@G1", "-n", "2", "-p", "1", "-r", "2", "-i", "3",
                                                      "-b", "8", "-l", "@LOGS"]))
    cases.append(run_case("err_zero_group_size", 2, 1, ["-f", "@G1", "-p", "1", "-u", "1", "-r", "2", "-l", "@LOGS"]))
    cases.append(run_case("err_missing_group_file", 2, 1, ["-f", "/nonexistent/g1", "-n", "1", "-p", "1", "-r",
                                                          "2"]))
    cases.append(run_case("err_all_in_group1_no_peer", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-u", "1", "-r",
                                                             "2", "-i", "1", "-b", "8", "-l", "@LOGS"],
                          host0="vm"))
    cases.append(run_case("odd_world_rank_without_peer", 3, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-u", "1", "-r",
                                                               "2", "-i", "1", "-b", "8", "-l", "@LOGS"]))
    # --- largest buffer the int -b accepts (mpi_perf.c:307) ---
    if os.environ.get("GOLDEN_BIG", "1") == "1":
        cases.append(run_case("max_int_buffer", 2, 1, ["-f", "@G1", "-n", "1", "-p", "1", "-u", "1", "-r", "2",
                                                       "-i", "1", "-b", "2147483647", "-l", "@LOGS"], timeout=600))
    meta = dict(
        generator="tests/golden/gen_golden.py",
        reference="/root/reference/mpi_perf.c compiled by `make -C oracle ref` (MPICH 3.3.2 ch3:nemesis from "
                  "/opt/conda, libuuid), run under mpiexec with oracle/ref_shim.c",
        checksum="oracle_checksum (oracle/mpx_oracle.c)",
        mpich=subprocess.run(["/opt/conda/bin/mpichversion"], capture_output=True, text=True).stdout.split("\n")[0],
    )
    with open(OUT, "w") as f:
        json.dump(dict(meta=meta, cases=cases), f, indent=1, sort_keys=True)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
