"""Hyper-parameter schedules over global timesteps.

Parity: reference rllib/utils/schedules/{piecewise_schedule,constant_schedule,linear_schedule,
exponential_schedule}.py and rllib/policy/torch_mixins.py (LearningRateSchedule /
EntropyCoeffSchedule: ``lr_schedule=[[t0, v0], [t1, v1], ...]`` interpolated linearly, the last
value held after the final endpoint)."""
from __future__ import annotations

from typing import Optional, Sequence


class Schedule:
    def value(self, t: float) -> float:
        raise NotImplementedError

    def __call__(self, t: float) -> float:
        return self.value(t)


class ConstantSchedule(Schedule):
    def __init__(self, v: float):
        self.v = float(v)

    def value(self, t):
        return self.v


class PiecewiseSchedule(Schedule):
    def __init__(self, endpoints: Sequence[Sequence[float]], outside_value: Optional[float] = None):
        pts = [(float(t), float(v)) for t, v in endpoints]
        if not pts:
            raise ValueError("PiecewiseSchedule needs at least one endpoint")
        if any(b[0] < a[0] for a, b in zip(pts, pts[1:])):
            raise ValueError("PiecewiseSchedule endpoints must be sorted by timestep")
        self.pts = pts
        self.outside = outside_value

    def value(self, t):
        pts = self.pts
        if t <= pts[0][0]:
            return pts[0][1] if self.outside is None else (pts[0][1] if t == pts[0][0] else self.outside)
        for (t0, v0), (t1, v1) in zip(pts, pts[1:]):
            if t0 <= t < t1:
                a = (t - t0) / (t1 - t0)
                return v0 + a * (v1 - v0)
        return pts[-1][1] if self.outside is None else self.outside


class LinearSchedule(Schedule):
    def __init__(self, schedule_timesteps: int, final_p: float, initial_p: float = 1.0):
        self.T, self.final, self.initial = float(schedule_timesteps), float(final_p), float(initial_p)

    def value(self, t):
        frac = min(float(t) / self.T, 1.0) if self.T > 0 else 1.0
        return self.initial + frac * (self.final - self.initial)


class ExponentialSchedule(Schedule):
    def __init__(self, schedule_timesteps: int, initial_p: float = 1.0, decay_rate: float = 0.1):
        self.T, self.initial, self.decay = float(schedule_timesteps), float(initial_p), float(decay_rate)

    def value(self, t):
        return self.initial * self.decay ** (float(t) / self.T)


class PolynomialSchedule(Schedule):
    """initial → final over `schedule_timesteps` along (1 - t/T)^power, then final."""

    def __init__(self, schedule_timesteps: int, final_p: float, initial_p: float = 1.0, power: float = 2.0):
        self.T, self.final, self.initial, self.power = float(schedule_timesteps), float(final_p), float(initial_p), \
            float(power)

    def value(self, t):
        frac = min(float(t), self.T) / self.T if self.T > 0 else 1.0
        return self.final + (self.initial - self.final) * (1.0 - frac) ** self.power


def make_schedule(spec, default: float) -> Schedule:
    """``None`` → constant default; list of [t, v] → piecewise; a Schedule passes through."""
    if spec is None:
        return ConstantSchedule(default)
    if isinstance(spec, Schedule):
        return spec
    return PiecewiseSchedule(spec)
