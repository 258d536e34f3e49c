"""`serve` command line. Parity: reference python/ray/serve/scripts.py (serve run <import_path>,
serve deploy <config.yaml> with the ServeApplicationSchema fields import_path / runtime_env /
deployments[name, num_replicas, route_prefix, user_config, max_concurrent_queries,
ray_actor_options], serve status, serve config, serve shutdown) against a running cluster
(`--address rmm://...` from `rmm start --head`).

    python -m ray_memory_management_amd.serve deploy app.yaml --address rmm://...
    python -m ray_memory_management_amd.serve status --address rmm://...
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time
from typing import List, Optional


def import_attr(path: str):
    """'pkg.module:attr' or 'pkg.module.attr' → the object."""
    if ":" in path:
        mod, attr = path.split(":", 1)
    else:
        mod, _, attr = path.rpartition(".")
    obj = importlib.import_module(mod)
    for part in attr.split("."):
        obj = getattr(obj, part)
    return obj


def _connect(address: Optional[str]):
    import ray_memory_management_amd as ray

    if not ray.is_initialized():
        ray.init(address=address or os.environ.get("RMM_ADDRESS") or "auto", namespace="serve")


def _apply_overrides(app, deployments: List[dict]):
    """Per-deployment option overrides from a config file, applied to the bound graph in place."""
    from ray_memory_management_amd.serve.api import Application

    by_name = {d["name"]: d for d in deployments or []}
    nodes = app._collect({}) if isinstance(app, Application) else {}
    for name, node in nodes.items():
        o = by_name.get(name)
        if not o:
            continue
        kw = {k: o[k] for k in ("num_replicas", "route_prefix", "user_config", "max_concurrent_queries",
                                "ray_actor_options", "autoscaling_config") if k in o}
        node.deployment = node.deployment.options(**kw)
    return app


def cmd_deploy(a) -> int:
    import yaml

    from ray_memory_management_amd import serve

    with open(a.config_file) as f:
        cfg = yaml.safe_load(f)
    if cfg.get("runtime_env", {}).get("working_dir"):
        sys.path.insert(0, cfg["runtime_env"]["working_dir"])
    _connect(a.address)
    app = import_attr(cfg["import_path"])
    app = _apply_overrides(app, cfg.get("deployments"))
    http = {"host": cfg.get("host", "127.0.0.1"), "port": int(cfg.get("port", a.port))}
    serve.start(detached=True, http_options=http)
    serve.run(app, host=http["host"], port=http["port"], route_prefix=cfg.get("route_prefix", "/"))
    print(json.dumps({"deployed": sorted(serve.list_deployments()), "http_port": serve.http_port()}), flush=True)
    return 0


def cmd_run(a) -> int:
    from ray_memory_management_amd import serve

    if a.app_dir:
        sys.path.insert(0, a.app_dir)
    _connect(a.address)
    app = import_attr(a.import_path)
    serve.start(detached=a.non_blocking, http_options={"host": a.host, "port": a.port})
    serve.run(app, host=a.host, port=a.port, route_prefix=a.route_prefix)
    print(json.dumps({"deployed": sorted(serve.list_deployments()), "http_port": serve.http_port()}), flush=True)
    if a.non_blocking:
        return 0
    try:
        while True:
            time.sleep(1.0)
    except KeyboardInterrupt:
        serve.shutdown()
    return 0


def cmd_status(a) -> int:
    from ray_memory_management_amd import serve

    _connect(a.address)
    print(json.dumps(serve.status(), default=str, indent=1), flush=True)
    return 0


def cmd_shutdown(a) -> int:
    from ray_memory_management_amd import serve

    _connect(a.address)
    serve.shutdown()
    print("serve shut down", flush=True)
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="serve")
    sub = p.add_subparsers(dest="cmd", required=True)
    d = sub.add_parser("deploy", help="deploy an application from a YAML config (detached)")
    d.add_argument("config_file")
    d.add_argument("--address", default=None)
    d.add_argument("--port", type=int, default=8000)
    d.set_defaults(fn=cmd_deploy)
    r = sub.add_parser("run", help="run an application given its import path")
    r.add_argument("import_path")
    r.add_argument("--address", default=None)
    r.add_argument("--host", default="127.0.0.1")
    r.add_argument("--port", type=int, default=8000)
    r.add_argument("--route-prefix", default="/")
    r.add_argument("--app-dir", default=None)
    r.add_argument("--non-blocking", action="store_true")
    r.set_defaults(fn=cmd_run)
    for name, fn in (("status", cmd_status), ("shutdown", cmd_shutdown)):
        x = sub.add_parser(name)
        x.add_argument("--address", default=None)
        x.set_defaults(fn=fn)
    a = p.parse_args(argv)
    return a.fn(a)
