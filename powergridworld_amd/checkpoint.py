"""Save / restore an environment's whole device state (SURVEY.md 5,
"Checkpoint / resume").

The reference's envs are not serialisable (only policies are checkpointed,
``examples/marl/rllib/heterogeneous/train.py:91-97``), and some of their state
silently persists across ``reset()`` -- the building's Kalman state ``x_k``
(``five_zone_rom_env.py:147-176``), the RegControl taps of the one OpenDSS
circuit (``opendss.py:36-39``).  Here all of it lives in device tensors and
plain attributes of the env objects, so ``state_dict()`` walks the env's
object tree (agents, components, the power-flow solver, the fused-step
buffers) and records

* every ``torch.Tensor`` it reaches (cloned; restored IN PLACE with ``copy_``:
  the native side holds raw pointers into these buffers, so they are never
  rebound),
* every ``torch.Generator`` (its state),
* the plain scalar attributes of the env objects (clocks, counters,
  timestamps) and small NumPy arrays (e.g. the EV's previous parking window);
  scalars inside dicts and lists are keys and indices, not state,

keyed by attribute path.  Cache-version counters, caches, the tensors a
solver keeps alive for an in-flight table upload and the solver's per-hour
tables (derived from the feeder and the hour, indexed on the host) are
skipped: they describe host-side tables, not the env's state; so are the {node: voltage} mappings,
views of the solver's output buffers (saved under the buffers' own names).  ``load_state_dict``
requires the same env configuration (same paths, shapes and dtypes) and
raises otherwise.

The voltage-history ring of ``MultiAgentEnv(record_history=True)`` (``_hist``,
[cap, nodes, N] on the device: gigabytes at large N) is NOT saved, like the
reference's own ``history`` lists it stands for
(``multiagent_env.py:129,191-194``): a restore empties it (write index 0,
lists cleared), so ``voltage_history()`` covers the steps after the restore.
"""
import datetime
import numbers
import warnings

import numpy as np
import torch

# caches, host-table keep-alives and the voltage mappings (views of buffers saved
# under their own names; MultiAgentEnv.load_state_dict re-arms them)
_SKIP_NAMES = ("version", "_ver", "cache", "_lib", "_memo", "keepalive", "voltages")
_SKIP_EXACT = ("history", "_hist", "_bv")  # the history lists and their device ring (emptied on load)
# the power-flow solver's per-hour tables (first-iteration / response / node
# records, predictor): derived data whose host-side index (_od_index,
# _pred_index) is not state -- a restore keeps the live tables and their index
# consistent (a checkpoint taken before a table rebuild would otherwise copy
# another hour's rows under the live index)
_SKIP_TABLES = ("_od_start", "_od_resp", "_od_vresp", "_od_qrec", "_pred_table", "_pred_sig", "_pred_meta",
                "_pred_grid",
                # the fused step's list of envs left to the solve: per-step scratch whose
                # counters pair with the live env's step parity (a restored count would not)
                "od_list", "od_count")
_SCALARS = (bool, numbers.Number, str, type(None), datetime.datetime, datetime.date, np.generic)


def _ours(obj):
    mod = type(obj).__module__ or ""
    return mod.startswith("powergridworld_amd")


def _skip(name):
    n = str(name).lower()
    return n in _SKIP_EXACT or n in _SKIP_TABLES or any(s in n for s in _SKIP_NAMES)


def _walk(obj, path, out, seen):
    """Append (path, owner, key, value) for every state leaf under obj.  `seen`
    holds the ancestors only: an object reachable under two names (a dict
    shared by the env and its solver) is recorded under both, so the paths do
    not depend on which name a given env instance happened to reach first."""
    if id(obj) in seen:
        return
    seen = seen | {id(obj)}
    if isinstance(obj, dict):
        items = [(k, v) for k, v in obj.items() if isinstance(k, (str, int))]
    elif isinstance(obj, (list, tuple)):
        items = list(enumerate(obj))
    elif _ours(obj) and hasattr(obj, "__dict__"):
        items = list(vars(obj).items())
    else:
        return
    for k, v in items:
        if _skip(k):
            continue
        p = "%s.%s" % (path, k) if path else str(k)
        if isinstance(v, torch.Tensor):
            # every path is recorded (a buffer reachable under two names is
            # saved and restored under both: the bindings may differ between
            # envs, e.g. before and after the first step); a view stands for
            # its base tensor
            if v._base is not None:
                out.append((p + "#base", None, None, v._base))
            else:
                out.append((p, obj, k, v))
        elif isinstance(v, torch.Generator):
            out.append((p, obj, k, v))
        elif isinstance(v, np.ndarray):
            # (containers hold tensors and objects; their scalars are indices and keys)
            if v.size <= 1 << 16 and not isinstance(obj, (list, tuple, dict)):
                out.append((p, obj, k, v))
        elif isinstance(v, _SCALARS) and not isinstance(obj, (list, tuple, dict)):
            out.append((p, obj, k, v))
        elif isinstance(v, (dict, list, tuple)) or (_ours(v) and hasattr(v, "__dict__")):
            _walk(v, p, out, seen)


def _leaves(env):
    out = []
    _walk(env, "", out, set())
    return out


def state_dict(env):
    """{path: value} of env's state: tensors cloned on their device, generator
    states, scalars and small arrays copied."""
    sd = {}
    for p, _, _, v in _leaves(env):
        if isinstance(v, torch.Tensor):
            sd[p] = v.detach().clone()
        elif isinstance(v, torch.Generator):
            sd[p] = ("generator", v.get_state().clone())
        elif isinstance(v, np.ndarray):
            sd[p] = v.copy()
        else:
            sd[p] = v
    return sd


def load_state_dict(env, sd, strict=False):
    """Restore a state_dict() of an env of the same configuration: tensors are
    copied into the env's own buffers, generators and attributes reset.  Paths
    present on one side only are attributes created lazily on the first step
    (derived per-step constants); strict=True refuses them instead."""
    leaves = _leaves(env)
    missing = [p for p, _, _, _ in leaves if p not in sd]
    known = {p for p, _, _, _ in leaves}
    extra = [p for p in sd if p not in known]
    if strict and (missing or extra):
        raise KeyError("state_dict does not match this env: missing %s, unexpected %s"
                       % (missing[:5], extra[:5]))
    tmiss = [p for p, _, _, v in leaves if p not in sd and isinstance(v, torch.Tensor)]
    textra = [p for p in extra if isinstance(sd[p], torch.Tensor)]
    if tmiss or textra:
        # lazily created buffers (first-step constants) exist on one side only;
        # say which, since a tensor left out is device state not restored
        warnings.warn("load_state_dict: tensors missing from the state_dict %s, not in this env %s"
                      % (tmiss[:8], textra[:8]), stacklevel=2)
    dev = getattr(env, "device", None)
    for p, owner, key, v in leaves:
        if p not in sd:
            continue
        s = sd[p]
        if isinstance(v, torch.Tensor):
            if not isinstance(s, torch.Tensor) or s.shape != v.shape or s.dtype != v.dtype:
                raise ValueError("state %s: expected %s %s" % (p, tuple(v.shape), v.dtype))
            v.copy_(s)
        elif isinstance(v, torch.Generator):
            v.set_state(s[1])
        else:
            if isinstance(s, torch.Tensor):
                # the live attribute is still unset (e.g. created on the first
                # step): bind a private copy on the env's device, never the
                # checkpoint's own tensor (the kernels get its pointer)
                val = s.detach().clone().to(dev if dev is not None else s.device)
            else:
                val = s.copy() if isinstance(s, np.ndarray) else s
            if isinstance(owner, dict):
                owner[key] = val
            else:
                setattr(owner, key, val)
    H = getattr(env, "_hist", None)
    if isinstance(H, dict):
        H["t"] = 0
    hist = getattr(env, "history", None)
    if isinstance(hist, dict):
        for v in hist.values():
            if isinstance(v, list):
                v.clear()
    return env
