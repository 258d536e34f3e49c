"""`serve deploy / status / shutdown` against a persistent head (reference
python/ray/serve/tests/test_cli.py): the deployed application outlives the deploying CLI process."""
import json
import os
import subprocess
import sys
import textwrap

import requests

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(mod, *args, timeout=180, extra_path=None):
    e = dict(os.environ)
    e["PYTHONPATH"] = os.pathsep.join([ROOT] + ([extra_path] if extra_path else []) + [e.get("PYTHONPATH", "")])
    return subprocess.run([sys.executable, "-m", mod, *args], capture_output=True, text=True, env=e, timeout=timeout)


def test_serve_deploy_status_shutdown(tmp_path):
    r = _run("ray_memory_management_amd.scripts", "start", "--head", "--num-cpus", "3",
             "--object-store-memory", str(128 << 20))
    assert r.returncode == 0, r.stderr + r.stdout
    addr = [w for w in r.stdout.split() if w.startswith("rmm://")][0]
    try:
        (tmp_path / "myapp.py").write_text(textwrap.dedent("""
            from ray_memory_management_amd import serve

            @serve.deployment(ray_actor_options={"num_cpus": 0})
            class Greeter:
                def __init__(self, greeting):
                    self.greeting = greeting

                async def __call__(self, request):
                    return {"msg": f"{self.greeting} {request.query_params.get('name', 'x')}"}

            app = Greeter.bind("hello")
        """))
        cfg = tmp_path / "serve.yaml"
        cfg.write_text(f"import_path: myapp:app\nport: 0\nruntime_env:\n  working_dir: {tmp_path}\n"
                       "deployments:\n  - name: Greeter\n    num_replicas: 2\n")
        r = _run("ray_memory_management_amd.serve", "deploy", str(cfg), "--address", addr, extra_path=str(tmp_path))
        assert r.returncode == 0, r.stdout + r.stderr
        info = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        assert info["deployed"] == ["Greeter"] and info["http_port"]
        # the deploying process has exited; the detached controller / proxy keep serving
        out = requests.get(f"http://127.0.0.1:{info['http_port']}/?name=amd", timeout=30)
        assert out.status_code == 200 and out.json() == {"msg": "hello amd"}
        r = _run("ray_memory_management_amd.serve", "status", "--address", addr)
        assert r.returncode == 0 and json.loads(r.stdout)["Greeter"]["num_replicas"] == 2, r.stdout + r.stderr
        r = _run("ray_memory_management_amd.serve", "shutdown", "--address", addr)
        assert r.returncode == 0, r.stderr
    finally:
        _run("ray_memory_management_amd.scripts", "stop", "--address", addr)
