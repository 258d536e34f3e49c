"""Command line interface: `python -m ray_memory_management_amd.scripts <command>` (or `bin/rmm`).

Parity: reference python/ray/scripts/scripts.py (start --head / stop / status / memory /
timeline / stack / microbenchmark / submit), experimental/state/state_cli.py (list / summary)
and dashboard/modules/job/cli.py (job submit / status / logs / stop / list / delete).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import tempfile
import time


def _connect(address=None):
    import ray_memory_management_amd as ray

    if not ray.is_initialized():
        ray.init(address=address or os.environ.get("RMM_ADDRESS") or "auto")
    return ray


def _session(address=None):
    from ray_memory_management_amd._private.worker import _find_session

    return _find_session(address or os.environ.get("RMM_ADDRESS") or "auto")


def cmd_start(a):
    import ray_memory_management_amd as ray
    from ray_memory_management_amd._private import worker as _w

    if not a.head:
        print("only `--head` is supported: every node of this runtime is started by the head (cluster_utils)")
        return 1
    res = json.loads(a.resources) if a.resources else None
    sc = {"gcs_storage_path": os.path.abspath(a.gcs_storage_path)} if a.gcs_storage_path else None
    ctx = ray.init(num_cpus=a.num_cpus, num_gpus=a.num_gpus, resources=res,
                   object_store_memory=a.object_store_memory, _persistent=True, _system_config=sc,
                   include_dashboard=a.include_dashboard, dashboard_host=a.dashboard_host,
                   dashboard_port=a.dashboard_port)
    sess = ctx["session_dir"]
    _w._head_proc = None  # detach: the head keeps running after this process exits
    _w._dashboard_proc = None  # the dashboard exits with the head
    ray.shutdown()
    if a.ray_client_server_port is not None:
        import subprocess
        import sys

        ready = os.path.join(sess, "client_server.json")
        log = open(os.path.join(sess, "logs", "ray_client_server.log"), "ab")
        subprocess.Popen([sys.executable, "-u", "-m", "ray_memory_management_amd.util.client.server", "--address",
                          f"rmm://{sess}", "--port", str(a.ray_client_server_port), "--ready-file", ready],
                         stdout=log, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, start_new_session=True)
        t0 = time.time()
        while not os.path.exists(ready) and time.time() - t0 < 60:
            time.sleep(0.05)
        if os.path.exists(ready):
            port = json.load(open(ready))["port"]
            print(f"  Ray Client server: ray://127.0.0.1:{port}")
    print(f"Started head. Address: rmm://{sess}\n  connect with ray.init(address='auto') or "
          f"RMM_ADDRESS=rmm://{sess}\n  stop with `rmm stop`")
    if ctx.dashboard_url:
        print(f"  dashboard: {ctx.dashboard_url}")
    return 0


def cmd_stop(a):
    try:
        sess = _session(a.address)
        info = json.load(open(os.path.join(sess, "session.json")))
    except (OSError, ValueError):
        print("no running cluster found")
        return 0
    pid = info.get("head_pid")
    try:
        os.kill(pid, signal.SIGKILL if a.force else signal.SIGTERM)
    except ProcessLookupError:
        pass
    t0 = time.time()
    while time.time() - t0 < a.grace_period:
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            break
        time.sleep(0.1)
    print(f"Stopped head (pid {pid})")
    return 0


def cmd_status(a):
    ray = _connect(a.address)
    tot, avail = ray.cluster_resources(), ray.available_resources()
    nodes = ray.nodes()
    print("======== Cluster status ========")
    print(f"Nodes: {len([n for n in nodes if n.get('Alive', True)])} alive")
    print("Resources:")
    for k in sorted(tot):
        if k.startswith("node:") or "_group_" in k:
            continue
        used = tot[k] - avail.get(k, 0)
        unit = ""
        if k in ("memory", "object_store_memory"):
            print(f"  {used / 2**30:.2f}/{tot[k] / 2**30:.2f} GiB {k}")
        else:
            print(f"  {used:g}/{tot[k]:g} {k}{unit}")
    from ray_memory_management_amd.autoscaler import sdk

    st = sdk.get_status()
    if st:
        print("======== Autoscaler ========")
        for t, n in sorted(st.get("active_nodes", {}).items()):
            print(f"  {n} {t}")
        print(f"  launches: {st.get('num_launches', 0)}  terminations: {st.get('num_terminations', 0)}")
        for d in st.get("demands", [])[:10]:
            print(f"  pending demand: {d}")
        for d in st.get("infeasible", [])[:10]:
            print(f"  infeasible: {d}")
        for e in st.get("events", [])[-5:]:
            print(f"  {e}")
    return 0


def cmd_memory(a):
    _connect(a.address)
    from ray_memory_management_amd import internal

    print(internal.memory_summary(stats_only=a.stats_only, units=a.units, num_entries=a.num_entries))
    return 0


def cmd_timeline(a):
    ray = _connect(a.address)
    path = a.output or os.path.join(tempfile.gettempdir(), f"rmm-timeline-{time.strftime('%Y-%m-%d_%H-%M-%S')}.json")
    ray.timeline(filename=path)
    print(f"Trace file written to {path} (open in chrome://tracing or ui.perfetto.dev)")
    return 0


def cmd_list(a):
    _connect(a.address)
    from ray_memory_management_amd.util import state

    fn = {"actors": state.list_actors, "tasks": state.list_tasks, "objects": state.list_objects,
          "nodes": state.list_nodes, "workers": state.list_workers, "jobs": state.list_jobs,
          "placement-groups": state.list_placement_groups}[a.resource]
    filters = []
    for f in a.filter or []:
        for op in ("!=", "="):
            if op in f:
                k, v = f.split(op, 1)
                filters.append((k.strip(), op, v.strip()))
                break
    rows = fn(filters=filters, limit=a.limit)
    if a.format == "json":
        print(json.dumps(rows, indent=1, default=str))
    else:
        for r in rows:
            print(json.dumps(r, default=str))
    return 0


def cmd_get(a):
    """`ray get <resource> <id>` (reference scripts.py ray_get): one state record as JSON."""
    _connect(a.address)
    from ray_memory_management_amd.util import state

    fn = {"actors": state.get_actor, "tasks": state.get_task, "objects": state.get_objects,
          "nodes": state.get_node, "workers": state.get_worker, "jobs": state.get_job,
          "placement-groups": state.get_placement_group}[a.resource]
    row = fn(a.id)
    if not row:
        print(f"{a.resource[:-1]} {a.id} not found", file=sys.stderr)
        return 1
    print(json.dumps(row, indent=1, default=str))
    return 0


def cmd_logs(a):
    """`ray logs` (reference scripts.py:1961): without a target, list the session's log files by category;
    with a file name / --actor-id / --task-id / --pid, print its last --tail lines (--follow keeps going)."""
    _connect(a.address)
    from ray_memory_management_amd.util import state

    if not (a.glob and any(c in a.glob for c in "*?[")) and (a.glob or a.actor_id or a.task_id or a.pid):
        for line in state.get_log(filename=a.glob, actor_id=a.actor_id, task_id=a.task_id, pid=a.pid,
                                  follow=a.follow, tail=a.tail):
            print(line, flush=a.follow)
        return 0
    for cat, files in sorted(state.list_logs(glob_filter=a.glob).items()):
        print(f"{cat}:")
        for f in files:
            print(f"  {f}")
    return 0


def cmd_global_gc(a):
    """`ray global-gc` (reference scripts.py): gc.collect() in every worker and driver."""
    _connect(a.address)
    from ray_memory_management_amd._private.internal_api import global_gc

    global_gc()
    print("Triggered gc.collect() on all workers.")
    return 0


def cmd_local_dump(a):
    """`ray local-dump` (reference scripts.py:2165, trimmed to what exists here): tar.gz of the session's
    logs, session.json and a state snapshot (actors / tasks / workers / nodes / memory summary)."""
    import io
    import tarfile

    sess = _session(a.address)
    out = a.output or os.path.join(tempfile.gettempdir(), f"rmm-local-dump-{int(time.time())}.tar.gz")
    with tarfile.open(out, "w:gz") as tar:
        logs = os.path.join(sess, "logs")
        if os.path.isdir(logs):
            tar.add(logs, arcname="logs")
        sj = os.path.join(sess, "session.json")
        if os.path.exists(sj):
            tar.add(sj, arcname="session.json")
        try:
            _connect(a.address)
            from ray_memory_management_amd._private.internal_api import memory_summary
            from ray_memory_management_amd.util import state

            snap = {"actors": state.list_actors(), "tasks": state.list_tasks(limit=2000),
                    "workers": state.list_workers(), "nodes": state.list_nodes(),
                    "memory_summary": memory_summary(stats_only=True)}
            data = json.dumps(snap, indent=1, default=str).encode()
            ti = tarfile.TarInfo("state.json")
            ti.size, ti.mtime = len(data), int(time.time())
            tar.addfile(ti, io.BytesIO(data))
        except Exception as e:  # noqa: BLE001 - a dead head still leaves its logs worth dumping
            print(f"state snapshot skipped: {e}", file=sys.stderr)
    print(out)
    return 0


def cmd_debug(a):
    """`ray debug` (reference scripts.py:202): list the active remote-pdb breakpoints registered in the
    cluster KV and attach to one (stdin/stdout relayed over its TCP socket)."""
    import socket

    _connect(a.address)
    from ray_memory_management_amd.util import rpdb

    bps = rpdb.list_breakpoints()
    if not bps:
        print("No active breakpoints.")
        return 0
    for i, b in enumerate(bps):
        print(f"{i}: pid {b['pid']} at {b['host']}:{b['port']} ({b['uuid']})")
    if a.list:
        return 0
    idx = a.index if a.index is not None else int(input("Enter breakpoint index or press enter to refresh: "))
    b = bps[idx]
    with socket.create_connection((b["host"], int(b["port"]))) as c:
        f = c.makefile("rw", buffering=1)
        import select

        while True:
            r, _, _ = select.select([c, sys.stdin], [], [])
            if c in r:
                data = c.recv(65536)
                if not data:
                    return 0
                sys.stdout.write(data.decode(errors="replace"))
                sys.stdout.flush()
            if sys.stdin in r:
                line = sys.stdin.readline()
                if not line:
                    return 0
                f.write(line)
                f.flush()


def _usage_stats_file():
    return os.path.join(os.path.expanduser("~"), ".rmm", "config.json")


def cmd_usage_stats(a):
    """`ray enable-usage-stats / disable-usage-stats`: recorded in ~/.rmm/config.json. Nothing is ever sent
    (no telemetry exists here); the flag is kept so scripts written for the reference run unchanged."""
    p = _usage_stats_file()
    os.makedirs(os.path.dirname(p), exist_ok=True)
    cfg = {}
    if os.path.exists(p):
        try:
            cfg = json.load(open(p))
        except ValueError:
            cfg = {}
    cfg["usage_stats"] = a.cmd == "enable-usage-stats"
    json.dump(cfg, open(p, "w"))
    print(f"Usage stats collection is {'enabled' if cfg['usage_stats'] else 'disabled'} (nothing is reported).")
    return 0


def cmd_serve(a):
    from ray_memory_management_amd.serve import scripts as serve_scripts

    return int(serve_scripts.main(a.serve_args) or 0)


def cmd_summary(a):
    _connect(a.address)
    from ray_memory_management_amd.util import state

    fn = {"tasks": state.summarize_tasks, "actors": getattr(state, "summarize_actors", state.summarize_tasks),
          "objects": getattr(state, "summarize_objects", state.summarize_tasks)}[a.resource]
    print(json.dumps(fn(), indent=1, default=str))
    return 0


def cmd_stack(a):
    """SIGUSR1 every worker of the local session: each dumps all thread stacks into its log."""
    sess = _session(a.address)
    info = json.load(open(os.path.join(sess, "session.json")))
    import psutil

    head = psutil.Process(info["head_pid"])
    n = 0
    for c in head.children(recursive=False):
        try:
            c.send_signal(signal.SIGUSR1)
            n += 1
        except psutil.Error:
            pass
    time.sleep(0.5)
    print(f"Dumped stacks of {n} worker processes into {os.path.join(sess, 'logs')}/worker-*.log")
    return 0


def cmd_microbenchmark(a):
    import ray_memory_management_amd as ray
    from ray_memory_management_amd._private import ray_perf

    ray.init(num_cpus=a.num_cpus, object_store_memory=a.object_store_memory)
    ray_perf.run(duration=a.duration, filter_pattern=a.filter)
    ray.shutdown()
    return 0


def cmd_job(a):
    from ray_memory_management_amd.job_submission import JobSubmissionClient

    c = JobSubmissionClient(a.address)
    if a.job_cmd == "submit":
        rt = json.loads(a.runtime_env_json) if a.runtime_env_json else {}
        if a.working_dir:
            rt["working_dir"] = a.working_dir
        sid = c.submit_job(entrypoint=" ".join(a.entrypoint), submission_id=a.submission_id, runtime_env=rt)
        print(f"Job '{sid}' submitted successfully")
        if not a.no_wait:
            for chunk in c.tail_job_logs(sid):
                print(chunk, end="")
            st = c.get_job_status(sid)
            print(f"\nJob '{sid}' {st.value}")
            return 0 if st.value == "SUCCEEDED" else 1
    elif a.job_cmd == "status":
        info = c.get_job_info(a.job_id)
        print(f"Status for job '{a.job_id}': {info.status.value}\nStatus message: {info.message}")
    elif a.job_cmd == "logs":
        if a.follow:
            for chunk in c.tail_job_logs(a.job_id):
                print(chunk, end="")
        else:
            print(c.get_job_logs(a.job_id), end="")
    elif a.job_cmd == "stop":
        c.stop_job(a.job_id)
        print(f"Job '{a.job_id}' stopped")
    elif a.job_cmd == "list":
        for j in c.list_jobs():
            print(json.dumps({"submission_id": j.submission_id, "status": j.status.value,
                              "entrypoint": j.entrypoint, "message": j.message}))
    elif a.job_cmd == "delete":
        c.delete_job(a.job_id)
        print(f"Job '{a.job_id}' deleted")
    return 0


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="rmm", description="ray_memory_management_amd cluster CLI")
    sub = p.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("start", help="start a persistent head node")
    s.add_argument("--head", action="store_true")
    s.add_argument("--num-cpus", type=int, default=None)
    s.add_argument("--num-gpus", type=int, default=None)
    s.add_argument("--include-dashboard", action="store_true")
    s.add_argument("--ray-client-server-port", type=int, default=None,
                   help="also start a Ray Client server (ray.init('ray://127.0.0.1:PORT'))")
    s.add_argument("--gcs-storage-path", default=None,
                   help="persist KV / detached actors / job history here; a head restarted with the same "
                        "path restores them")
    s.add_argument("--dashboard-host", default="127.0.0.1")
    s.add_argument("--dashboard-port", type=int, default=8265)
    s.add_argument("--resources", default=None, help="JSON dict of custom resources")
    s.add_argument("--object-store-memory", type=int, default=None)
    s.set_defaults(fn=cmd_start)
    s = sub.add_parser("stop", help="stop the head started by `rmm start`")
    s.add_argument("--address", default=None)
    s.add_argument("-f", "--force", action="store_true")
    s.add_argument("-g", "--grace-period", type=float, default=10)
    s.set_defaults(fn=cmd_stop)
    for name, fn in (("status", cmd_status), ("timeline", cmd_timeline), ("stack", cmd_stack)):
        s = sub.add_parser(name)
        s.add_argument("--address", default=None)
        if name == "timeline":
            s.add_argument("--output", default=None)
        s.set_defaults(fn=fn)
    s = sub.add_parser("memory", help="object store usage and objects")
    s.add_argument("--address", default=None)
    s.add_argument("--stats-only", action="store_true")
    s.add_argument("--units", default="MB", choices=["B", "KB", "MB", "GB"])
    s.add_argument("--num-entries", type=int, default=50)
    s.set_defaults(fn=cmd_memory)
    s = sub.add_parser("list", help="state API listing")
    s.add_argument("resource", choices=["actors", "tasks", "objects", "nodes", "workers", "jobs",
                                        "placement-groups"])
    s.add_argument("--address", default=None)
    s.add_argument("-f", "--filter", action="append")
    s.add_argument("--limit", type=int, default=100)
    s.add_argument("--format", default="table", choices=["table", "json"])
    s.set_defaults(fn=cmd_list)
    s = sub.add_parser("get", help="one state record by id")
    s.add_argument("resource", choices=["actors", "tasks", "objects", "nodes", "workers", "jobs",
                                        "placement-groups"])
    s.add_argument("id")
    s.add_argument("--address", default=None)
    s.set_defaults(fn=cmd_get)
    s = sub.add_parser("logs", help="list the session's log files, or print one")
    s.add_argument("glob", nargs="?", default=None, help="file name, or a glob filter for the listing")
    s.add_argument("--actor-id", default=None)
    s.add_argument("--task-id", default=None)
    s.add_argument("--pid", type=int, default=None)
    s.add_argument("--tail", type=int, default=1000)
    s.add_argument("-f", "--follow", action="store_true")
    s.add_argument("--address", default=None)
    s.set_defaults(fn=cmd_logs)
    s = sub.add_parser("global-gc", help="gc.collect() in every worker and driver")
    s.add_argument("--address", default=None)
    s.set_defaults(fn=cmd_global_gc)
    s = sub.add_parser("local-dump", help="tar.gz of the session's logs and a state snapshot")
    s.add_argument("--address", default=None)
    s.add_argument("--output", default=None)
    s.set_defaults(fn=cmd_local_dump)
    s = sub.add_parser("debug", help="list / attach to remote-pdb breakpoints")
    s.add_argument("--address", default=None)
    s.add_argument("--list", action="store_true")
    s.add_argument("--index", type=int, default=None)
    s.set_defaults(fn=cmd_debug)
    for name in ("enable-usage-stats", "disable-usage-stats"):
        s = sub.add_parser(name)
        s.set_defaults(fn=cmd_usage_stats)
    s = sub.add_parser("serve", help="serve deploy / run / status / shutdown")
    s.add_argument("serve_args", nargs=argparse.REMAINDER)
    s.set_defaults(fn=cmd_serve)
    s = sub.add_parser("summary")
    s.add_argument("resource", choices=["tasks", "actors", "objects"])
    s.add_argument("--address", default=None)
    s.set_defaults(fn=cmd_summary)
    s = sub.add_parser("microbenchmark", help="core microbenchmarks (ray_perf)")
    s.add_argument("--duration", type=float, default=2.0)
    s.add_argument("--filter", default="")
    s.add_argument("--num-cpus", type=int, default=None)
    s.add_argument("--object-store-memory", type=int, default=None)
    s.set_defaults(fn=cmd_microbenchmark)
    j = sub.add_parser("job", help="job submission")
    jsub = j.add_subparsers(dest="job_cmd", required=True)
    x = jsub.add_parser("submit")
    x.add_argument("--address", default=None)
    x.add_argument("--submission-id", default=None)
    x.add_argument("--working-dir", default=None)
    x.add_argument("--runtime-env-json", default=None)
    x.add_argument("--no-wait", action="store_true")
    x.add_argument("entrypoint", nargs=argparse.REMAINDER)
    for name in ("status", "logs", "stop", "delete"):
        x = jsub.add_parser(name)
        x.add_argument("job_id")
        x.add_argument("--address", default=None)
        if name == "logs":
            x.add_argument("-f", "--follow", action="store_true")
    x = jsub.add_parser("list")
    x.add_argument("--address", default=None)
    j.set_defaults(fn=cmd_job)
    return p


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    if getattr(a, "entrypoint", None) and a.entrypoint[:1] == ["--"]:
        a.entrypoint = a.entrypoint[1:]
    return int(a.fn(a) or 0)


if __name__ == "__main__":
    sys.exit(main())
