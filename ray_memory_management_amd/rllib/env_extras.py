"""More of the ``rllib.env`` namespace: EnvContext, GroupAgentsWrapper, ExternalMultiAgentEnv,
RemoteBaseEnv, PolicyClient / PolicyServerInput, and gated wrappers for third-party env suites.

Parity: reference rllib/env/{env_context.py, wrappers/group_agents_wrapper.py,
external_multi_agent_env.py, remote_base_env.py, policy_client.py, policy_server_input.py,
wrappers/{dm_env_wrapper, dm_control_wrapper, pettingzoo_env, unity3d_env}.py}.

PolicyServerInput / PolicyClient speak JSON over HTTP (observations and actions as nested
lists): the server runs inside a rollout worker as its ``input`` (``config["input"] = lambda
ioctx: PolicyServerInput(ioctx, "127.0.0.1", 9900)``), external applications drive episodes through
PolicyClient; the server computes actions with the worker's policy ("remote" inference) or records
the client's own actions (``log_action``), postprocesses finished trajectories (GAE when the policy
has a value function) and hands SampleBatches to the algorithm like any sampler.
"""
from __future__ import annotations

import json
import queue
import threading
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional

import numpy as np

from ray_memory_management_amd.rllib.base_env import _DUMMY_AGENT, BaseEnv, ExternalEnv
from ray_memory_management_amd.rllib.sample_batch import SampleBatch


class EnvContext(dict):
    """The env_config dict plus the worker / vector slot the env runs in."""

    def __init__(self, env_config: Dict, worker_index: int = 0, vector_index: int = 0, remote: bool = False,
                 num_workers: Optional[int] = None, recreated_worker: bool = False):
        super().__init__(env_config or {})
        self.worker_index, self.vector_index, self.remote = worker_index, vector_index, remote
        self.num_workers, self.recreated_worker = num_workers, recreated_worker

    def copy_with_overrides(self, env_config=None, worker_index=None, vector_index=None, remote=None,
                            num_workers=None, recreated_worker=None) -> "EnvContext":
        return EnvContext(self if env_config is None else env_config,
                          self.worker_index if worker_index is None else worker_index,
                          self.vector_index if vector_index is None else vector_index,
                          self.remote if remote is None else remote,
                          self.num_workers if num_workers is None else num_workers,
                          self.recreated_worker if recreated_worker is None else recreated_worker)


class GroupAgentsWrapper:
    """Present groups of agents of a MultiAgentEnv as single agents (tuple obs / actions, summed
    rewards), e.g. for QMIX."""

    def __init__(self, env, groups: Dict[str, List], obs_space=None, act_space=None):
        self.env, self.groups = env, groups
        self.agent_id_to_group = {a: g for g, agents in groups.items() for a in agents}
        self.observation_space = obs_space if obs_space is not None else getattr(env, "observation_space", None)
        self.action_space = act_space if act_space is not None else getattr(env, "action_space", None)

    def _group(self, items: Dict, agg=None):
        out: Dict = {}
        for g, agents in self.groups.items():
            vals = [items[a] for a in agents if a in items]
            if vals:
                out[g] = agg(vals) if agg else vals
        for a, v in items.items():
            if a not in self.agent_id_to_group:
                out[a] = v
        return out

    def reset(self):
        return self._group(self.env.reset())

    def step(self, action_dict):
        flat = {}
        for g, a in action_dict.items():
            if g in self.groups:
                for agent, act in zip(self.groups[g], a):
                    flat[agent] = act
            else:
                flat[g] = a
        obs, rew, done, info = self.env.step(flat)
        dones = self._group({k: v for k, v in done.items() if k != "__all__"}, all)
        dones["__all__"] = done.get("__all__", all(dones.values()))
        return (self._group(obs), self._group(rew, lambda v: float(np.sum(v))), dones,
                self._group(info, lambda v: {"_group_info": v}))


class ExternalMultiAgentEnv(ExternalEnv):
    """ExternalEnv whose observations / actions / rewards are {agent_id: value} dicts."""

    def get_action(self, episode_id: str, observation_dict: Dict) -> Dict:
        return super().get_action(episode_id, observation_dict)

    def log_returns(self, episode_id: str, reward_dict: Dict, info_dict=None, multiagent_done_dict=None) -> None:
        ep = self._episodes[episode_id]
        if not isinstance(ep.reward, dict):
            ep.reward = {}
        for k, v in reward_dict.items():
            ep.reward[k] = ep.reward.get(k, 0.0) + float(v)

    def _publish(self, ep, obs, done: bool):
        with self._ready:
            self._outbox[ep.episode_id] = (obs, ep.reward if isinstance(ep.reward, dict) else {}, done,
                                           ep.off_policy_action)
            ep.reward, ep.off_policy_action = {}, None
            self._ready.notify_all()


class RemoteBaseEnv(BaseEnv):
    """Each sub-env runs in its own actor; ``poll`` returns the envs whose step finished."""

    def __init__(self, make_env, num_envs: int, multiagent: bool = False, remote_env_batch_wait_ms: int = 0,
                 existing_envs=None, worker=None):
        import ray_memory_management_amd as ray

        class _EnvActor:
            def __init__(self, mk, i):
                self.env = mk(i)

            def reset(self):
                return self.env.reset()

            def step(self, a):
                return self.env.step(a)

            def spaces(self):
                return self.env.observation_space, self.env.action_space

        cls = ray.remote(_EnvActor)
        self.multiagent = multiagent
        self.wait_s = remote_env_batch_wait_ms / 1000.0
        self.actors = [cls.remote(make_env, i) for i in range(num_envs)]
        self.observation_space, self.action_space = ray.get(self.actors[0].spaces.remote())
        self.pending = {a.reset.remote(): (i, True) for i, a in enumerate(self.actors)}

    def poll(self):
        import ray_memory_management_amd as ray

        ready, _ = ray.wait(list(self.pending), num_returns=1)
        if self.wait_s > 0:
            more, _ = ray.wait(list(self.pending), num_returns=len(self.pending), timeout=self.wait_s)
            ready = list(dict.fromkeys(list(ready) + list(more)))
        obs, rew, done, info = {}, {}, {}, {}
        for r in ready:
            i, is_reset = self.pending.pop(r)
            res = ray.get(r)
            if is_reset:
                o, rr, d, inf = res, ({} if self.multiagent else 0.0), False, {}
            else:
                o, rr, d, inf = res
            if self.multiagent:
                obs[i], rew[i], done[i], info[i] = o, rr, (d if isinstance(d, dict) else {"__all__": d}), inf
            else:
                obs[i], rew[i] = {_DUMMY_AGENT: o}, {_DUMMY_AGENT: rr}
                done[i], info[i] = {_DUMMY_AGENT: d, "__all__": d}, {_DUMMY_AGENT: inf}
        return obs, rew, done, info, {}

    def send_actions(self, action_dict):
        for i, acts in action_dict.items():
            a = acts if self.multiagent else acts[_DUMMY_AGENT]
            self.pending[self.actors[i].step.remote(a)] = (i, False)

    def try_reset(self, env_id=None):
        self.pending[self.actors[env_id].reset.remote()] = (env_id, True)
        return None

    def stop(self):
        import ray_memory_management_amd as ray

        for a in self.actors:
            try:
                ray.kill(a)
            except Exception:
                pass


# ============================================================================ policy server / client
def _jsonable(x):
    if isinstance(x, np.ndarray):
        return x.tolist()
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    if isinstance(x, dict):
        return {str(k): _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    return x


class _ServerEnv(ExternalEnv):
    def run(self):
        threading.Event().wait()  # episodes are driven by the HTTP handler threads


class PolicyServerInput:
    """InputReader fed by external applications over HTTP (see module docstring)."""

    def __init__(self, ioctx=None, address: str = "127.0.0.1", port: int = 9900, idle_timeout: float = 3.0,
                 policy=None, rollout_fragment_length: Optional[int] = None):
        worker = getattr(ioctx, "worker", None)
        self.policy = policy if policy is not None else (worker.get_policy() if worker is not None else None)
        if self.policy is None:
            raise ValueError("PolicyServerInput needs a policy (ioctx.worker or policy=...)")
        cfg = getattr(ioctx, "config", None) or getattr(worker, "config", None) or {}
        self.fragment = int(rollout_fragment_length or cfg.get("rollout_fragment_length", 200) or 200)
        self.env = _ServerEnv(self.policy.action_space, self.policy.observation_space)
        self.env.start()
        self.base = self.env.to_base_env()
        self.batches: "queue.Queue" = queue.Queue()
        self.idle_timeout = idle_timeout
        self._builders: Dict[str, Dict[str, list]] = {}
        self._last: Dict[str, tuple] = {}
        self._stop = False
        server_self = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_POST(self):
                n = int(self.headers.get("Content-Length", 0))
                req = json.loads(self.rfile.read(n) or b"{}")
                try:
                    resp = {"ok": True, "result": _jsonable(server_self._handle(req))}
                except Exception as e:  # reported to the client
                    resp = {"ok": False, "error": repr(e)}
                body = json.dumps(resp).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.httpd = ThreadingHTTPServer((address, port), Handler)
        self.address = f"http://{address}:{self.httpd.server_address[1]}"
        threading.Thread(target=self.httpd.serve_forever, daemon=True, name="policy-server").start()
        threading.Thread(target=self._sample_loop, daemon=True, name="policy-server-sampler").start()

    # ------------------------------------------------------------------ HTTP commands
    def _handle(self, req: Dict):
        cmd = req.get("command")
        env = self.env
        if cmd == "START_EPISODE":
            return env.start_episode(req.get("episode_id"), req.get("training_enabled", True))
        if cmd == "GET_ACTION":
            return env.get_action(req["episode_id"], np.asarray(req["observation"]))
        if cmd == "LOG_ACTION":
            env.log_action(req["episode_id"], np.asarray(req["observation"]), req["action"])
            return None
        if cmd == "LOG_RETURNS":
            env.log_returns(req["episode_id"], req["reward"], req.get("info"))
            return None
        if cmd == "END_EPISODE":
            env.end_episode(req["episode_id"], np.asarray(req["observation"]))
            return None
        if cmd == "GET_WEIGHTS":
            return {k: np.asarray(v).tolist() for k, v in self.policy.get_weights().items()}
        raise ValueError(f"unknown command {cmd!r}")

    # ------------------------------------------------------------------ sampling
    def _flush(self, eid: str, done: bool):
        cols = self._builders.pop(eid, None)
        if not cols or not cols[SampleBatch.OBS]:
            return
        b = SampleBatch({k: np.asarray(v) for k, v in cols.items()})
        if hasattr(self.policy, "value") and SampleBatch.VF_PREDS in b:
            from ray_memory_management_amd.rllib.evaluation.postprocessing import compute_gae_for_sample_batch

            b = compute_gae_for_sample_batch(self.policy, b)
        elif hasattr(self.policy, "postprocess_trajectory"):
            b = self.policy.postprocess_trajectory(b)
        self.batches.put(b)

    def _sample_loop(self):
        while not self._stop:
            try:
                obs, rew, done, info, off = self.base.poll()
            except TimeoutError:
                continue
            actions, compute = {}, []
            for eid, ob in obs.items():
                o = ob[_DUMMY_AGENT]
                r = rew[eid][_DUMMY_AGENT]
                d = bool(done[eid]["__all__"])
                last = self._last.pop(eid, None)
                if last is not None:
                    cols = self._builders.setdefault(eid, {})
                    lo, la, extra, t = last
                    row = {SampleBatch.OBS: lo, SampleBatch.ACTIONS: la, SampleBatch.REWARDS: float(r),
                           SampleBatch.DONES: d, SampleBatch.NEXT_OBS: np.asarray(o),
                           SampleBatch.EPS_ID: abs(hash(eid)) % (1 << 31), SampleBatch.T: t, **extra}
                    for k, v in row.items():
                        cols.setdefault(k, []).append(v)
                    if d or len(cols[SampleBatch.OBS]) >= self.fragment:
                        self._flush(eid, d)
                if d:
                    continue
                t = (last[3] + 1) if last is not None else 0
                if eid in off:
                    a = off[eid][_DUMMY_AGENT]
                    self._last[eid] = (np.asarray(o), a, self._logged_extras(np.asarray(o), a), t)
                    actions[eid] = {_DUMMY_AGENT: a}
                else:
                    compute.append((eid, np.asarray(o), t))
            if compute:
                a, _, extra = self.policy.compute_actions([c[1] for c in compute], explore=True)
                for j, (eid, o, t) in enumerate(compute):
                    ex = {k: np.asarray(v)[j] for k, v in (extra or {}).items() if v is not None}
                    self._last[eid] = (o, a[j], ex, t)
                    actions[eid] = {_DUMMY_AGENT: a[j]}
            if actions:
                self.base.send_actions(actions)

    def _logged_extras(self, obs, action) -> Dict:
        """Policy columns for an action the application chose (off-policy): the policy's logp of
        THAT action, its value estimate and its logits, so logged rows carry the same columns as
        served ones."""
        pol = self.policy
        model, dist_cls = getattr(pol, "model", None), getattr(pol, "dist_class", None)
        if model is None or dist_cls is None:
            return {}
        import torch

        with torch.no_grad():
            logits, v = model(torch.as_tensor(obs[None], device=getattr(pol, "device", "cpu")))
            d = dist_cls(logits.float())
            lp = d.logp(torch.as_tensor(np.asarray([action]), device=logits.device))
        return {SampleBatch.ACTION_LOGP: float(lp[0]), SampleBatch.VF_PREDS: float(v.reshape(-1)[0]),
                SampleBatch.ACTION_DIST_INPUTS: logits[0].float().cpu().numpy()}

    def next(self) -> SampleBatch:
        from ray_memory_management_amd.rllib.sample_batch import concat_samples

        out = [self.batches.get()]
        while True:
            try:
                out.append(self.batches.get_nowait())
            except queue.Empty:
                break
        return concat_samples(out)

    def stop(self):
        self._stop = True
        self.httpd.shutdown()


class PolicyClient:
    """Client of a PolicyServerInput (inference_mode "remote": the server picks actions)."""

    def __init__(self, address: str, inference_mode: str = "remote", update_interval: float = 10.0):
        if inference_mode not in ("remote", "local"):
            raise ValueError("inference_mode must be 'remote' or 'local'")
        self.address = address if address.startswith("http") else f"http://{address}"
        self.inference_mode = inference_mode
        self.local_policy = None

    def _send(self, data: Dict):
        body = json.dumps(_jsonable(data)).encode()
        req = urllib.request.Request(self.address, data=body, headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=120) as r:
            resp = json.loads(r.read())
        if not resp.get("ok"):
            raise RuntimeError(f"policy server error: {resp.get('error')}")
        return resp.get("result")

    def start_episode(self, episode_id: Optional[str] = None, training_enabled: bool = True) -> str:
        return self._send({"command": "START_EPISODE", "episode_id": episode_id, "training_enabled": training_enabled})

    def get_action(self, episode_id: str, observation):
        if self.inference_mode == "local" and self.local_policy is not None:
            a = self.local_policy.compute_single_action(observation)
            self.log_action(episode_id, observation, a)
            return a
        return self._send({"command": "GET_ACTION", "episode_id": episode_id, "observation": observation})

    def log_action(self, episode_id: str, observation, action) -> None:
        self._send({"command": "LOG_ACTION", "episode_id": episode_id, "observation": observation, "action": action})

    def log_returns(self, episode_id: str, reward: float, info=None, multiagent_done_dict=None) -> None:
        self._send({"command": "LOG_RETURNS", "episode_id": episode_id, "reward": reward, "info": info})

    def end_episode(self, episode_id: str, observation) -> None:
        self._send({"command": "END_EPISODE", "episode_id": episode_id, "observation": observation})

    def update_policy_weights(self) -> None:
        """Local inference: pull the server policy's weights into the client's copy."""
        if self.local_policy is None:
            raise ValueError("set client.local_policy (a Policy) for local inference")
        import torch

        w = self._send({"command": "GET_WEIGHTS"})
        self.local_policy.set_weights({k: torch.as_tensor(np.asarray(v)) for k, v in w.items()})


# ============================================================================ gated third-party suites
def _gated(name: str, lib: str):
    class _Gated:
        def __init__(self, *a, **kw):
            raise ImportError(f"{name} wraps `{lib}`, which is not installed in this environment")

    _Gated.__name__ = _Gated.__qualname__ = name
    return _Gated


DMEnv = _gated("DMEnv", "dm_env")
DMCEnv = _gated("DMCEnv", "dm_control")
PettingZooEnv = _gated("PettingZooEnv", "pettingzoo")
ParallelPettingZooEnv = _gated("ParallelPettingZooEnv", "pettingzoo")
Unity3DEnv = _gated("Unity3DEnv", "mlagents_envs")
