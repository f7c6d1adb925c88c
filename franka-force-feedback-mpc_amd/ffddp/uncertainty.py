"""Benchmark uncertainty profile of the closed loop (src/run/uncertainty_profiles.py).

``actuation_uncertainty`` draws an actuation gain a and bias b once, delays
and perturbs the observations the controller sees (state noise, noisy torque
measurement with a first-order filter) and replaces the applied command by
a * (delayed command) + b + noise.  Same numpy Generator stream as the
reference (seeded PCG64, draws in the same order), so a run with the same
seed sees the same perturbations (tests/test_closed_loop.py pins it against
outputs the reference wrote).
"""
from __future__ import annotations

import dataclasses
from collections import deque
from dataclasses import dataclass
from typing import Optional

import numpy as np


@dataclass
class UncertaintyProfileConfig:
    """uncertainty_profiles.py:12-30."""

    a_min: float = 0.95
    a_max: float = 1.05
    b_min: float = -0.1
    b_max: float = 0.1
    sigma_q: float = 5.0e-4
    sigma_dq: float = 2.0e-3
    sigma_tau: float = 5.0e-2
    delta_obs_cycles: int = 2
    delta_cmd_s: float = 1.0e-3
    seed: int = 0


def config_for_scenario(scenario: str, seed: int = 0) -> Optional[UncertaintyProfileConfig]:
    """Only actuation_uncertainty carries an injected profile (uncertainty_profiles.py:33-53)."""
    if str(scenario).strip().lower() != "actuation_uncertainty":
        return None
    return UncertaintyProfileConfig(seed=int(seed))


_ARRAY_FIELDS = ("q", "dq", "tau_meas", "tau_meas_filt", "tau_meas_act", "tau_meas_act_filt", "tau_cmd", "tau_act",
                 "tau_constraint", "tau_total", "tau_bias", "f_contact_world", "ee_pos", "ee_quat", "J_pos", "J_rot",
                 "ee_vel")


def copy_observation(obs):
    """Deep copy of the array fields of an Observation dataclass."""
    kw = {}
    for f in _ARRAY_FIELDS:
        if hasattr(obs, f):
            v = getattr(obs, f)
            kw[f] = None if v is None else np.asarray(v, dtype=float).copy()
    return dataclasses.replace(obs, **kw)


class ScenarioUncertaintyInjector:
    """uncertainty_profiles.py:84-161, draw for draw."""

    def __init__(self, dt: float, nu: int, config: UncertaintyProfileConfig, tau_lpf_alpha: float = 0.2):
        self.dt = float(max(dt, 1.0e-9))
        self.nu = int(nu)
        self.cfg = config
        self.rng = np.random.default_rng(int(config.seed))
        self.a = float(self.rng.uniform(float(config.a_min), float(config.a_max)))
        self.b = float(self.rng.uniform(float(config.b_min), float(config.b_max)))
        self.obs_delay_cycles_1khz = int(max(config.delta_obs_cycles, 0))
        # the observation delay is specified in 1 kHz cycles; convert to control steps
        self.obs_delay_steps = int(max(np.round(self.obs_delay_cycles_1khz * 1.0e-3 / self.dt), 0))
        self.cmd_delay_steps = int(max(np.round(float(config.delta_cmd_s) / self.dt), 0))
        self._obs_hist: deque = deque(maxlen=self.obs_delay_steps + 1)
        self._cmd_hist: deque = deque([np.zeros(self.nu) for _ in range(self.cmd_delay_steps + 1)],
                                      maxlen=self.cmd_delay_steps + 1)
        self._tau_hat_filt = np.zeros(self.nu)
        self._tau_lpf_alpha = float(np.clip(tau_lpf_alpha, 0.0, 1.0))

    def meta(self) -> dict:
        return {"a": float(self.a), "b": float(self.b), "sigma_q": float(self.cfg.sigma_q),
                "sigma_dq": float(self.cfg.sigma_dq), "sigma_tau": float(self.cfg.sigma_tau),
                "delta_obs_cycles_1khz": int(self.obs_delay_cycles_1khz), "delta_obs_steps": int(self.obs_delay_steps),
                "delta_cmd_steps": int(self.cmd_delay_steps), "delta_cmd_s": float(self.cfg.delta_cmd_s),
                "seed": int(self.cfg.seed)}

    def _tau_hat(self) -> np.ndarray:
        noise = self.rng.normal(0.0, float(self.cfg.sigma_tau), size=self.nu)
        return self.a * np.asarray(self._cmd_hist[0], dtype=float).reshape(self.nu) + self.b + noise

    def observation_for_controller(self, obs):
        cur = copy_observation(obs)
        if not self._obs_hist:
            self._obs_hist.extend(copy_observation(cur) for _ in range(self.obs_delay_steps + 1))
        else:
            self._obs_hist.append(cur)
        out = copy_observation(self._obs_hist[0])
        out.q = out.q + self.rng.normal(0.0, float(self.cfg.sigma_q), size=self.nu)
        out.dq = out.dq + self.rng.normal(0.0, float(self.cfg.sigma_dq), size=self.nu)
        th = self._tau_hat()
        a = self._tau_lpf_alpha
        self._tau_hat_filt = (1.0 - a) * self._tau_hat_filt + a * th
        out.tau_meas = th.copy()
        out.tau_meas_filt = self._tau_hat_filt.copy()
        out.tau_meas_act = th.copy()
        out.tau_meas_act_filt = self._tau_hat_filt.copy()
        return out

    def command_for_plant(self, tau_cmd_nominal) -> np.ndarray:
        self._cmd_hist.append(np.asarray(tau_cmd_nominal, dtype=float).reshape(self.nu).copy())
        return self._tau_hat()


class BatchedUncertaintyInjector:
    """ScenarioUncertaintyInjector for many instances at once (the closed-loop
    fleet's actuation_uncertainty scenario): each instance keeps its own
    seeded Generator and draws, in the scalar injector's order, the same
    numbers -- per tick 7 + 7 + 7 normals for the observation (q, dq, torque
    measurement) and 7 for the command -- pre-drawn a chunk of ticks at a time
    (a Generator's normals are one stream however many a call asks for), and
    the delay lines are ring buffers over the batch.  Only the fields the
    fleet reads are produced: the delayed noisy (q, dq) and the applied
    command.  Bit-identical to per-instance ScenarioUncertaintyInjector calls
    (tests/test_closed_loop.py)."""

    CHUNK = 256  # ticks of normals drawn per Generator call

    def __init__(self, dt: float, nu: int, configs, tau_lpf_alpha: float = 0.2):
        self.nu = int(nu)
        self.dt = float(max(dt, 1.0e-9))
        self.cfgs = list(configs)
        self.B = len(self.cfgs)
        c0 = self.cfgs[0] if self.cfgs else UncertaintyProfileConfig()
        for c in self.cfgs:  # one delay / noise model (they differ by seed only)
            if dataclasses.replace(c, seed=0) != dataclasses.replace(c0, seed=0):
                raise ValueError("BatchedUncertaintyInjector: configs may differ by seed only")
        self.rngs = [np.random.default_rng(int(c.seed)) for c in self.cfgs]
        ab = [(float(r.uniform(float(c.a_min), float(c.a_max))), float(r.uniform(float(c.b_min), float(c.b_max))))
              for r, c in zip(self.rngs, self.cfgs)]
        self.a = np.array([x[0] for x in ab])
        self.b = np.array([x[1] for x in ab])
        self.obs_delay_steps = int(max(np.round(int(max(c0.delta_obs_cycles, 0)) * 1.0e-3 / self.dt), 0))
        self.cmd_delay_steps = int(max(np.round(float(c0.delta_cmd_s) / self.dt), 0))
        self.sig = (float(c0.sigma_q), float(c0.sigma_dq), float(c0.sigma_tau))
        self._obs = None  # [D+1][B][14] ring of (q, dq); slot _oi is the oldest
        self._oi = 0
        self._cmd = np.zeros((self.cmd_delay_steps + 1, self.B, self.nu))
        self._ci = 0
        self._z = np.zeros((self.B, 0, 4 * self.nu))
        self._zi = 0

    def _normals(self):
        """this tick's 28 normals per instance: q, dq, tau (observation), tau (command)"""
        if self._zi >= self._z.shape[1]:
            self._z = np.stack([r.standard_normal(self.CHUNK * 4 * self.nu).reshape(self.CHUNK, 4 * self.nu)
                                for r in self.rngs])
            self._zi = 0
        z = self._z[:, self._zi]
        self._zi += 1
        return z

    def _tau_hat(self, z7):
        return self.a[:, None] * self._cmd[self._ci] + self.b[:, None] + (0.0 + self.sig[2] * z7)

    def observation_for_controller(self, q, dq):
        """(q, dq) [B][nu] -> the delayed, noisy (q, dq) the controllers see."""
        nu = self.nu
        cur = np.concatenate([np.asarray(q, float), np.asarray(dq, float)], 1)
        if self._obs is None:
            self._obs = np.repeat(cur[None], self.obs_delay_steps + 1, 0)
            self._oi = 0
        else:  # deque(maxlen).append: the oldest slot takes the newest entry
            self._obs[self._oi] = cur
            self._oi = (self._oi + 1) % (self.obs_delay_steps + 1)
        old = self._obs[self._oi]
        self._z_tick = z = self._normals()
        qo = old[:, :nu] + (0.0 + self.sig[0] * z[:, :nu])
        dqo = old[:, nu:] + (0.0 + self.sig[1] * z[:, nu:2 * nu])
        self._tau_hat(z[:, 2 * nu:3 * nu])  # the torque measurement's draw (the fleet does not read it)
        return qo, dqo

    def command_for_plant(self, tau_cmd):
        """tau_cmd [B][nu] -> the applied torques a * (delayed command) + b + noise."""
        self._cmd[self._ci] = np.asarray(tau_cmd, float)
        self._ci = (self._ci + 1) % (self.cmd_delay_steps + 1)
        return self._tau_hat(self._z_tick[:, 3 * self.nu:])
