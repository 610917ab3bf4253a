"""Hydra-free composition of the reference's YAML configs (cfg/config.yaml + cfg/task/<Task>.yaml).

The reference composes its configs with hydra/OmegaConf and registers four resolvers
(isaacgymenvs/__init__.py:8-11):

    eq               ${eq:a,b}                a.lower() == b.lower()
    contains         ${contains:a,b}          a.lower() in b.lower()
    if               ${if:pred,a,b}           a if pred else b
    resolve_default  ${resolve_default:d,x}   d if x == '' else x

Neither hydra nor omegaconf is installed here, so this module restates the part the task configs use:
YAML loading (PyYAML, safe loader), the ``defaults:`` task choice, hydra-style ``key=value`` overrides,
absolute (``${a.b}``) and relative (``${..x}``: one leading dot is the node holding the value, each
further dot one level up) interpolations, string interpolation inside longer strings, and the four
resolvers with nested interpolations, quoted and bare arguments.  ``omegaconf_to_dict`` of the composed
``cfg.task`` is what ``isaacgymenvs.make`` hands to the task (isaacgymenvs/__init__.py:35-38), and it is
what :func:`task_config_from_yaml` returns.

Built-in defaults (no YAML directory needed) stay in :mod:`migym.configs`; a user's own YAMLs (a copy of
the reference's ``cfg/`` tree, edited) load through :func:`compose` / :func:`task_config_from_yaml`.
"""
from __future__ import annotations

import copy
import os
import re
from typing import Any, Dict, List, Optional

import yaml

RESOLVERS = {
    "eq": lambda x, y: str(x).lower() == str(y).lower(),
    "contains": lambda x, y: str(x).lower() in str(y).lower(),
    "if": lambda pred, a, b: a if pred else b,
    "resolve_default": lambda default, arg: default if arg == "" else arg,
}

class ConfigError(ValueError):
    pass


def load_yaml(path_or_text: str) -> dict:
    """A YAML mapping from a file path or a YAML string (safe loader only)."""
    if os.path.exists(path_or_text):
        with open(path_or_text) as f:
            data = yaml.safe_load(f)
    else:
        data = yaml.safe_load(path_or_text)
    return {} if data is None else data


# ------------------------------------------------------------------------------------ interpolation
def _find_close(s: str, i: int) -> int:
    """index of the '}' closing the '${' that starts at s[i]"""
    depth, j, quote = 0, i, None
    while j < len(s):
        c = s[j]
        if quote:
            if c == quote:
                quote = None
        elif c in "'\"":
            quote = c
        elif s.startswith("${", j):
            depth += 1
            j += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return j
        j += 1
    raise ConfigError(f"unterminated interpolation in {s!r}")


def _split_args(s: str) -> List[str]:
    """split resolver arguments at top-level commas"""
    out, depth, quote, cur = [], 0, None, ""
    i = 0
    while i < len(s):
        c = s[i]
        if quote:
            cur += c
            if c == quote:
                quote = None
        elif c in "'\"":
            quote = c
            cur += c
        elif s.startswith("${", i):
            depth += 1
            cur += "${"
            i += 2
            continue
        elif c == "}":
            depth -= 1
            cur += c
        elif c == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += c
        i += 1
    out.append(cur)
    return [a.strip() for a in out]


class _Resolver:
    def __init__(self, root: dict):
        self.root = root
        self.active = set()

    def lookup(self, ref: str, here: List[str]):
        if ref.startswith("."):
            nd = len(ref) - len(ref.lstrip("."))
            base = here[:-1]               # the node holding the value
            up = nd - 1
            if up > len(base):
                raise ConfigError(f"relative interpolation ${{{ref}}} at {'.'.join(here)} climbs above the root")
            path = base[:len(base) - up] if up else list(base)
            rest = ref[nd:]
        else:
            path, rest = [], ref
        if rest:
            path = path + rest.split(".")
        node: Any = self.root
        for k in path:
            if isinstance(node, dict) and k in node:
                node = node[k]
            elif isinstance(node, list) and k.isdigit() and int(k) < len(node):
                node = node[int(k)]
            else:
                raise ConfigError(f"interpolation ${{{ref}}} at {'.'.join(here)}: key {'.'.join(path)!r} not found")
        return self.value(node, path)

    def arg(self, a: str, here: List[str]):
        if len(a) >= 2 and a[0] == a[-1] and a[0] in "'\"":
            return self.string(a[1:-1], here)
        if a.startswith("${") and _find_close(a, 0) == len(a) - 1:
            return self.expr(a[2:-1], here)
        if "${" in a:
            return self.string(a, here)
        if a == "":
            return ""
        return yaml.safe_load(a)

    def expr(self, body: str, here: List[str]):
        m = re.match(r"^\s*([A-Za-z_][A-Za-z0-9_]*)\s*:(.*)$", body, re.S)
        if m and m.group(1) in RESOLVERS:
            args = [self.arg(a, here) for a in _split_args(m.group(2))]
            return RESOLVERS[m.group(1)](*args)
        if m and not body.strip().startswith("."):
            raise ConfigError(f"unknown resolver {m.group(1)!r} in ${{{body}}}")
        return self.lookup(body.strip(), here)

    def string(self, s: str, here: List[str]):
        """a string with interpolations: one whole-string interpolation keeps its type"""
        if s.startswith("${") and _find_close(s, 0) == len(s) - 1:
            return self.expr(s[2:-1], here)
        out, i = "", 0
        while True:
            j = s.find("${", i)
            if j < 0:
                return out + s[i:]
            k = _find_close(s, j)
            out += s[i:j] + str(self.expr(s[j + 2:k], here))
            i = k + 1

    def value(self, node, path: List[str]):
        key = tuple(path)
        if isinstance(node, dict):
            return {k: self.value(v, path + [str(k)]) for k, v in node.items()}
        if isinstance(node, list):
            return [self.value(v, path + [str(i)]) for i, v in enumerate(node)]
        if isinstance(node, str) and "${" in node:
            if key in self.active:
                raise ConfigError(f"interpolation cycle at {'.'.join(path)}")
            self.active.add(key)
            try:
                return self.string(node, path)
            finally:
                self.active.discard(key)
        return node


def resolve(cfg: dict, lazy: bool = False) -> dict:
    """every interpolation of ``cfg`` resolved (a new dict; ``OmegaConf.to_container(resolve=True)``).
    lazy: OmegaConf resolves on access, so a top-level key whose interpolation cannot resolve (the root
    config's ``wandb_name: ${train...}`` without the train group) is kept unresolved instead of failing."""
    r = _Resolver(cfg)
    if not lazy:
        return r.value(cfg, [])
    out = {}
    for k, v in cfg.items():
        try:
            out[k] = r.value(v, [str(k)])
        except ConfigError:
            out[k] = copy.deepcopy(v)
    return out


# ------------------------------------------------------------------------------------ composition
def _parse_override(ov: str):
    if "=" not in ov:
        raise ConfigError(f"override {ov!r} is not key=value")
    k, v = ov.split("=", 1)
    k = k.strip().lstrip("+")
    return k, (yaml.safe_load(v) if v.strip() != "" else "")


def _set_path(cfg: dict, dotted: str, v):
    node = cfg
    parts = dotted.split(".")
    for p in parts[:-1]:
        node = node.setdefault(p, {})
    node[parts[-1]] = v


def compose(cfg_dir: str, task: Optional[str] = None, overrides: Optional[List[str]] = None) -> dict:
    """``hydra.compose(config_name="config", overrides=[...])`` for the reference's layout: cfg_dir/config.yaml
    with its ``defaults`` task choice (or ``task``), cfg_dir/task/<Task>.yaml under the key ``task``,
    hydra-style overrides (``task=Humanoid``, ``num_envs=64``, ``task.env.episodeLength=200``), then every
    interpolation resolved.  The train / pbt groups are not composed (not on this path)."""
    root = load_yaml(os.path.join(cfg_dir, "config.yaml"))
    defaults = root.pop("defaults", []) or []
    root.pop("hydra", None)
    choice = None
    for d in defaults:
        if isinstance(d, dict) and "task" in d:
            choice = d["task"]
    ovs = [_parse_override(o) for o in (overrides or [])]
    for k, v in ovs:
        if k == "task":
            choice = v
    if task is not None:
        choice = task
    if not choice:
        raise ConfigError("no task chosen (defaults list or task=...)")
    tpath = os.path.join(cfg_dir, "task", f"{choice}.yaml")
    if not os.path.exists(tpath):
        raise ConfigError(f"no task config {tpath}")
    root["task"] = load_yaml(tpath)
    for k, v in ovs:
        if k != "task":
            _set_path(root, k, v)
    out = resolve(root, lazy=True)
    out["task"] = _Resolver(root).value(root["task"], ["task"])   # the task group must resolve completely
    return out


def task_config_from_yaml(task: str, cfg_dir: str, num_envs=None, sim_device: str = "cuda:0",
                          pipeline: str = "gpu", overrides: Optional[List[str]] = None) -> Dict[str, Any]:
    """``cfg.task`` as ``isaacgymenvs.make`` builds it from YAML (isaacgymenvs/__init__.py:31-38): compose with
    the device / pipeline choices, then ``env.numEnvs = num_envs`` when given."""
    ovs = [f"sim_device={sim_device}", f"pipeline={pipeline}"] + list(overrides or [])
    cfg = compose(cfg_dir, task=task, overrides=ovs)
    t = copy.deepcopy(cfg["task"])
    if num_envs not in (None, ""):
        t["env"]["numEnvs"] = int(num_envs)
    return t


def task_config_from_file(path: str, root: Optional[dict] = None, num_envs=None) -> Dict[str, Any]:
    """One task YAML on its own (a user file): its relative interpolations resolve against ``root`` (the
    reference's config.yaml defaults for the keys the task files use when omitted)."""
    from .configs import ROOT_DEFAULTS
    base = dict(ROOT_DEFAULTS)
    base.update({"num_envs": "" if num_envs is None else int(num_envs)})
    base.update(root or {})
    base["task"] = load_yaml(path)
    t = resolve(base)["task"]
    if num_envs not in (None, ""):
        t["env"]["numEnvs"] = int(num_envs)
    return t
