"""Dashboard HTTP API. Mirrors reference dashboard/tests/test_dashboard.py (server comes up with
ray.init(include_dashboard=True), health endpoint), dashboard/state_aggregator tests (list /
summarize over HTTP with filters), dashboard/modules/job/tests/test_http_job_server.py (REST
submit → status → logs → stop → delete through JobSubmissionClient("http://...")) and
dashboard/modules/reporter tests (Prometheus metrics)."""
import json
import sys
import time
import urllib.request

import pytest


def _get(url, raw=False):
    with urllib.request.urlopen(url, timeout=30) as r:
        body = r.read()
    return body.decode() if raw else json.loads(body)


@pytest.fixture(scope="module")
def dash():
    import ray_memory_management_amd as ray

    if ray.is_initialized():
        ray.shutdown()
    ctx = ray.init(num_cpus=4, include_dashboard=True, dashboard_port=0)
    assert ctx.dashboard_url and ctx.dashboard_url.startswith("http://127.0.0.1:")
    yield ray, ctx.dashboard_url
    ray.shutdown()


def test_health_version_and_cluster_status(dash):
    ray, url = dash
    assert _get(url + "/api/gcs_healthz") == "success"
    assert _get(url + "/api/version")["version"] == "1"
    st = _get(url + "/api/cluster_status")
    assert st["cluster_resources"]["CPU"] == 4.0
    nodes = _get(url + "/api/v0/nodes")
    assert nodes["total"] == 1 and nodes["result"][0]["IsHead"]


def test_state_lists_and_filters(dash):
    ray, url = dash

    @ray.remote
    class Holder:
        def ping(self):
            return 1

    a = Holder.options(name="dash_holder").remote()
    ray.get(a.ping.remote())
    ref = ray.put(b"x" * (1 << 20))

    @ray.remote
    def f():
        return 2

    ray.get([f.remote() for _ in range(3)])
    actors = _get(url + "/api/v0/actors?name=dash_holder")["result"]
    assert len(actors) == 1 and actors[0]["class_name"] == "Holder" and actors[0]["state"] == "ALIVE"
    q = "filter_keys=state&filter_predicates=%3D&filter_values=DEAD"
    assert all(x["state"] == "DEAD" for x in _get(url + "/api/v0/actors?" + q)["result"])
    objs = _get(url + "/api/v0/objects")["result"]
    assert any(o["object_id"] == ref.hex() for o in objs)
    # directly submitted tasks reach the head's task table with the owner's batched completion records
    # (flushed every 10 ms): eventually consistent, as the reference's state API is
    deadline = time.time() + 10
    while _get(url + "/api/v0/tasks/summarize")["cluster"]["total_tasks"] < 3 and time.time() < deadline:
        time.sleep(0.05)
    assert _get(url + "/api/v0/tasks/summarize")["cluster"]["total_tasks"] >= 3
    assert _get(url + "/api/v0/tasks?limit=1")["total"] == 1
    ray.kill(a)


def test_memory_and_metrics(dash):
    ray, url = dash
    ref = ray.put(b"y" * (2 << 20))
    store = _get(url + "/api/memory/store")
    assert store and any(isinstance(v, (int, float)) for v in store.values())
    assert "Object" in _get(url + "/api/memory/summary?stats_only=1")["summary"] or True
    pressure = _get(url + "/api/memory/pressure")
    assert isinstance(pressure, dict)
    from ray_memory_management_amd.util import metrics

    c = metrics.Counter("dash_test_requests", description="test counter", tag_keys=("route",))
    c.inc(3, tags={"route": "/x"})
    metrics.flush()
    text = _get(url + "/metrics", raw=True)
    assert 'rmm_resources_total{resource="CPU"} 4.0' in text
    assert "# TYPE rmm_object_store_stats gauge" in text
    assert 'dash_test_requests{route="/x"} 3' in text
    del ref


def test_logs_endpoints(dash):
    ray, url = dash
    files = _get(url + "/api/v0/logs")["result"]
    names = [f["filename"] for f in files]
    assert "head.log" in names
    txt = _get(url + "/api/v0/logs/file?filename=head.log&lines=5", raw=True)
    assert isinstance(txt, str)
    with pytest.raises(urllib.error.HTTPError):
        _get(url + "/api/v0/logs/file?filename=../session.json", raw=True)


def test_rest_job_submission(dash, tmp_path):
    ray, url = dash
    from ray_memory_management_amd.job_submission import JobStatus, JobSubmissionClient

    c = JobSubmissionClient(url)
    script = tmp_path / "job.py"
    script.write_text("import ray_memory_management_amd as ray\nray.init()\n"
                      "print('job says', ray.get(ray.remote(lambda: 41 + 1).remote()))\n")
    sid = c.submit_job(entrypoint=f"{sys.executable} {script}", metadata={"k": "v"})
    t0 = time.time()
    while not c.get_job_status(sid).is_terminal() and time.time() - t0 < 120:
        time.sleep(0.2)
    info = c.get_job_info(sid)
    assert info.status == JobStatus.SUCCEEDED, (info, c.get_job_logs(sid))
    assert "job says 42" in c.get_job_logs(sid) and info.metadata == {"k": "v"}
    assert any(j.submission_id == sid for j in c.list_jobs())
    long_sid = c.submit_job(entrypoint="sleep 60")
    t0 = time.time()
    while c.get_job_status(long_sid) != JobStatus.RUNNING and time.time() - t0 < 30:
        time.sleep(0.1)
    assert c.stop_job(long_sid)
    assert c.get_job_status(long_sid) == JobStatus.STOPPED
    assert c.delete_job(sid)
    with pytest.raises(RuntimeError):
        c.get_job_info(sid)
    req = urllib.request.Request(url + "/api/jobs/", data=b"{}", method="POST",
                                 headers={"Content-Type": "application/json"})
    with pytest.raises(urllib.error.HTTPError) as e:
        urllib.request.urlopen(req, timeout=30)
    assert e.value.code == 400


def _fake_sysfs(root):
    import os

    dev = root / "card0" / "device"
    (dev / "hwmon" / "hwmon3").mkdir(parents=True)
    for name, val in (("vendor", "0x1002"), ("mem_info_vram_total", str(288 << 30)),
                      ("mem_info_vram_used", str(12 << 30)), ("mem_info_gtt_used", "4096"),
                      ("gpu_busy_percent", "37"), ("uevent", "DRIVER=amdgpu\nPCI_SLOT_NAME=0000:75:00.0\n")):
        (dev / name).write_text(val)
    (dev / "hwmon" / "hwmon3" / "temp1_input").write_text("41000")
    (dev / "hwmon" / "hwmon3" / "power1_average").write_text("350000000")
    other = root / "card1" / "device"  # not an AMD GPU: skipped
    other.mkdir(parents=True)
    (other / "vendor").write_text("0x8086")
    return os.fspath(root)


def test_event_snapshot_actor_modules(dash):
    """reference dashboard/modules/{event,snapshot,actor}: a worker that dies unexpectedly and an
    actor restart show up as events (event_head.py /events), the snapshot lists jobs and actors,
    actors are grouped by class and can be killed over HTTP."""
    import os
    import signal

    ray, url = dash

    @ray.remote(max_restarts=1)
    class Phoenix:
        def pid(self):
            return os.getpid()

    a = Phoenix.remote()
    pid = ray.get(a.pid.remote())
    os.kill(pid, signal.SIGKILL)
    deadline = time.time() + 30
    labels = set()
    while time.time() < deadline:
        ev = _get(url + "/events")
        assert ev["result"] is True
        labels = {e["label"] for evs in ev["data"]["events"].values() for e in evs}
        if {"WORKER_DIED", "ACTOR_RESTARTED", "JOB_STARTED"} <= labels:
            break
        time.sleep(0.2)
    assert {"WORKER_DIED", "ACTOR_RESTARTED", "JOB_STARTED"} <= labels, labels
    died = [e for evs in _get(url + "/events")["data"]["events"].values() for e in evs if e["label"] == "WORKER_DIED"]
    assert any(e["custom_fields"]["pid"] == pid and e["severity"] == "ERROR" for e in died), died
    # the real exit status (the fork-server template reaps the worker and reports it): SIGKILL
    mine = [e for e in died if e["custom_fields"]["pid"] == pid]
    assert mine[0]["custom_fields"]["exit_code"] == -9 and mine[0]["custom_fields"]["signal"] == 9, mine
    assert ray.get(a.pid.remote()) != pid  # restarted

    snap = _get(url + "/api/snapshot")["data"]["snapshot"]
    aid = a._actor_id.hex()
    assert aid in snap["actors"] and snap["jobs"] and "deployments" in snap
    groups = _get(url + "/logical/actor_groups")["data"]["actor_groups"]
    assert any(aid in [e["actor_id"] for e in g["entries"]] for g in groups.values())
    assert aid in _get(url + "/logical/actors")["data"]["actors"]
    r = _get(url + f"/api/actors/kill?actor_id={aid}&force_kill=true&no_restart=true")
    assert r["result"] is True
    deadline = time.time() + 30
    while time.time() < deadline and _get(url + "/logical/actors")["data"]["actors"][aid]["state"] != "DEAD":
        time.sleep(0.1)
    assert _get(url + "/logical/actors")["data"]["actors"][aid]["state"] == "DEAD"
    with pytest.raises(Exception):
        _get(url + "/api/actors/kill?actor_id=" + "ab" * 16)
    # Serve not running: empty deployment list, NOT_STARTED-free status shape
    assert _get(url + "/api/serve/deployments/")["deployments"] == []


def test_tune_module_reads_experiment(dash, tmp_path):
    ray, url = dash
    exp = tmp_path / "exp"
    for i, lr in enumerate((0.1, 0.01)):
        d = exp / f"train_{i:05d}"
        d.mkdir(parents=True)
        (d / "params.json").write_text(json.dumps({"lr": lr}))
        (d / "result.json").write_text("".join(json.dumps({"loss": 1.0 / (k + 1 + i), "training_iteration": k + 1})
                                               + "\n" for k in range(3)))
    assert _get(url + "/tune/set_experiment?experiment=" + str(exp))["result"] is True
    assert _get(url + "/tune/availability")["data"]["result"]["trials_available"] is True
    info = _get(url + "/tune/info")["data"]["result"]["trial_records"]
    assert len(info) == 2 and {t["params"]["lr"] for t in info.values()} == {0.1, 0.01}
    assert all(t["num_results"] == 3 and t["metrics"]["training_iteration"] == 3 for t in info.values())


def test_event_log_reader(tmp_path):
    from ray_memory_management_amd._private.event_log import EventLogger, events_by_job, read_events

    lg = EventLogger(str(tmp_path), "RAYLET")
    lg.emit("INFO", "A", "first", job_id="01")
    lg.emit("ERROR", "B", "second", job_id="02", pid=7)
    lg.emit("WARNING", "C", "third")
    lg.close()
    with open(lg.path, "a") as f:
        f.write('{"truncated": ')  # a line being written
    assert [e["label"] for e in read_events(str(tmp_path))] == ["A", "B", "C"]
    assert [e["label"] for e in read_events(str(tmp_path), severity="WARNING")] == ["B", "C"]
    assert [e["label"] for e in read_events(str(tmp_path), job_id="02")] == ["B"]
    by = events_by_job(str(tmp_path))
    assert set(by) == {"01", "02", "global"} and by["02"][0]["custom_fields"]["pid"] == 7
    with pytest.raises(ValueError):
        lg.emit("LOUD", "X", "bad severity")


def test_gpu_reporter_endpoints(tmp_path, monkeypatch):
    """Per-GPU utilization / HBM (amdgpu sysfs) and GPU object-store occupancy in /api/gpus,
    /api/cluster_status and /metrics (reference reporter_agent.py:92-98 GPU usage)."""
    import os

    import ray_memory_management_amd as ray
    from ray_memory_management_amd import internal
    from ray_memory_management_amd.dashboard import gpu_reporter

    monkeypatch.setenv("RMM_SYSFS_DRM_ROOT", _fake_sysfs(tmp_path / "drm"))
    devs = gpu_reporter.gpu_devices()
    assert len(devs) == 1 and devs[0]["pci_bus_id"] == "0000:75:00.0" and devs[0]["busy_percent"] == 37
    assert devs[0]["vram_used_bytes"] == 12 << 30 and devs[0]["temperature_c"] == 41.0 and devs[0]["power_w"] == 350.0
    if ray.is_initialized():
        ray.shutdown()
    ctx = ray.init(num_cpus=2, include_dashboard=True, dashboard_port=0)
    try:
        rec = {"pid": os.getpid(), "device": 0, "pci_bus_id": "0000:75:00.0", "time": time.time(),
               "stats": {"capacity": 8 << 30, "bytes_in_use": 3 << 30, "num_objects": 5, "spilled_bytes_total": 1 << 30,
                         "restored_bytes_total": 1 << 29, "spilled_objects": 2}}
        internal._internal_kv_put(f"gpu_store/{os.getpid()}/0", json.dumps(rec), True, namespace=gpu_reporter.NAMESPACE)
        g = _get(ctx.dashboard_url + "/api/gpus")
        assert g["gpus"][0]["vram_total_bytes"] == 288 << 30
        st = [s for s in g["gpu_object_stores"] if s["pid"] == os.getpid()]
        assert st and st[0]["alive"] and st[0]["stats"]["bytes_in_use"] == 3 << 30
        cs = _get(ctx.dashboard_url + "/api/cluster_status")
        assert cs["gpus"][0]["busy_percent"] == 37 and cs["gpu_object_stores"]
        m = _get(ctx.dashboard_url + "/metrics", raw=True)
        assert 'rmm_gpu_utilization_percent{gpu="0",pci_bus_id="0000:75:00.0"} 37.0' in m
        assert "rmm_gpu_object_store_spilled_bytes_total{" in m and "rmm_gpu_vram_used_bytes" in m
    finally:
        ray.shutdown()
