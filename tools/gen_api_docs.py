#!/usr/bin/env python3
"""Public API reference -> ``docs/API.md`` (the reference's ``npm run docs`` / ``grunt docs``:
jsdoc over ``lib/hlsjs-p2p-wrapper.js`` and ``lib/hlsjs-p2p-bundle.js``, ``package.json:21``,
``Gruntfile.js:113-116``).

Generated from the docstrings and signatures of the pure-Python sources (the Cython-compiled
modules are bypassed so the output does not depend on the build):

    python tools/gen_api_docs.py            # rewrite docs/API.md
    python tools/gen_api_docs.py --check    # exit 1 if docs/API.md is stale (CI / tests)
"""
from __future__ import annotations

import inspect
import os
import sys
from pathlib import Path

os.environ["HLSJS_P2P_PURE"] = "1"  # document the sources, not whichever build is present
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
OUT = REPO / "docs" / "API.md"

# (section, import path, object name) in reading order: the public surface of SURVEY §A.5
# and the contracts of §2.3 that an integrator touches
SURFACE = [
    ("Bundle", "hlsjs_p2p_wrapper_amd.api.bundle", "Hls"),
    ("Wrapper facade", "hlsjs_p2p_wrapper_amd.api.wrapper", "HlsjsP2PWrapper"),
    ("Session orchestrator", "hlsjs_p2p_wrapper_amd.api.wrapper_private", "HlsjsP2PWrapperPrivate"),
    ("Fragment loader", "hlsjs_p2p_wrapper_amd.integration.p2p_loader", "p2p_loader_generator"),
    ("Player bridge", "hlsjs_p2p_wrapper_amd.integration.player_interface", "PlayerInterface"),
    ("Segment identity", "hlsjs_p2p_wrapper_amd.models.track_view", "TrackView"),
    ("Segment identity", "hlsjs_p2p_wrapper_amd.models.segment_view", "SegmentView"),
    ("Media map", "hlsjs_p2p_wrapper_amd.models.media_map", "MediaMap"),
    ("Peer agent", "hlsjs_p2p_wrapper_amd.agent.peer_agent", "PeerAgent"),
    ("Swarm node", "hlsjs_p2p_wrapper_amd.agent.node", "SwarmNode"),
    ("Swarm node", "hlsjs_p2p_wrapper_amd.agent.node", "node_for_config"),
    ("Media engine", "hlsjs_p2p_wrapper_amd.player.hls", "Hls"),
    ("Media engine", "hlsjs_p2p_wrapper_amd.player.media", "MediaElement"),
    ("Events", "hlsjs_p2p_wrapper_amd.player.events", "Events"),
    ("Events", "hlsjs_p2p_wrapper_amd.player.events", "ErrorTypes"),
    ("Events", "hlsjs_p2p_wrapper_amd.player.events", "ErrorDetails"),
    ("xhrSetup sandbox", "hlsjs_p2p_wrapper_amd.utils.xhr", "extractInfoFromXhrSetup"),
    ("Statics", "hlsjs_p2p_wrapper_amd.utils.statics", "inheritStaticPropertiesReadOnly"),
    ("Metrics", "hlsjs_p2p_wrapper_amd.utils.metrics", "MetricsServer"),
    ("Fleet (player processes per GPU)", "hlsjs_p2p_wrapper_amd.parallel.fleet", "FleetServer"),
    ("Fleet (player processes per GPU)", "hlsjs_p2p_wrapper_amd.parallel.fleet", "RemoteNode"),
    ("Fleet (player processes per GPU)", "hlsjs_p2p_wrapper_amd.parallel.fleet", "player_main"),
    ("Network CDN", "hlsjs_p2p_wrapper_amd.net.http", "enable_network"),
    ("Network CDN", "hlsjs_p2p_wrapper_amd.net.network", "HttpOrigin"),
    ("Checkpoint", "hlsjs_p2p_wrapper_amd.agent.checkpoint", "save_cache"),
    ("Checkpoint", "hlsjs_p2p_wrapper_amd.agent.checkpoint", "load_cache"),
]


class _Raw:
    """Renders as its text: unquoted string annotations, class defaults by name."""

    def __init__(self, text: str) -> None:
        self.text = text

    def __repr__(self) -> str:
        return self.text


def _clean(sig: inspect.Signature, drop_first: bool = False) -> str:
    params = []
    for i, prm in enumerate(sig.parameters.values()):
        if drop_first and i == 0:
            continue
        ann, dflt = prm.annotation, prm.default
        if isinstance(ann, str):
            ann = _Raw(ann)
        if inspect.isclass(dflt) and dflt is not inspect.Parameter.empty:
            dflt = _Raw(dflt.__name__)
        params.append(prm.replace(annotation=ann, default=dflt))
    ret = sig.return_annotation
    ret = _Raw(ret) if isinstance(ret, str) else ret
    return str(sig.replace(parameters=params, return_annotation=ret))


def _sig(obj, drop_first: bool = False) -> str:
    try:
        return _clean(inspect.signature(obj), drop_first)
    except (TypeError, ValueError):
        return "(...)"


def _doc(obj, first_paragraph: bool = False) -> str:
    d = inspect.getdoc(obj) or ""
    if first_paragraph:
        d = d.split("\n\n", 1)[0]
    return d.strip()


def _members(cls):
    """Public methods / properties defined on ``cls`` itself; aliases (one function bound under
    two names, e.g. ``isLive`` / ``is_live``) collapse into one row."""
    out, seen = [], {}
    for name, attr in cls.__dict__.items():
        if name.startswith("_"):
            continue
        if isinstance(attr, property):
            kind, fn = "property", attr
        elif isinstance(attr, (staticmethod, classmethod)):
            kind, fn = "method", attr.__func__
        elif inspect.isfunction(attr):
            kind, fn = "method", attr
        else:
            continue
        if id(fn) in seen:
            seen[id(fn)][3].append(name)
            continue
        row = [kind, name, fn, []]
        seen[id(fn)] = row
        out.append(row)
    return out


def _takes_self(fn) -> bool:
    params = list(inspect.signature(fn).parameters)
    return bool(params) and params[0] in ("self", "cls")


def _ctor(cls) -> str:
    """Constructor signature: ``__new__`` when the class builds something else (the bundle),
    else ``__init__``; ``self`` / ``cls`` dropped."""
    fn = cls.__dict__.get("__new__") or cls.__dict__.get("__init__")
    if fn is None:
        return ""
    fn = fn.__func__ if isinstance(fn, staticmethod) else fn
    sig = inspect.signature(fn)
    return _clean(sig.replace(return_annotation=inspect.Signature.empty), drop_first=True)


def _enum_values(cls):
    vals = [(k, v) for k, v in vars(cls).items() if not k.startswith("_") and isinstance(v, (str, int))]
    return vals


def render() -> str:
    import importlib

    lines = ["# API reference", "",
             "Generated by `tools/gen_api_docs.py` from the package docstrings (the analog of the",
             "reference's `npm run docs`); `python tools/gen_api_docs.py --check` fails when this file is",
             "stale. Behavioural parity with the reference is mapped in `docs/PARITY.md`.", ""]
    section = None
    for sec, mod_name, name in SURFACE:
        mod = importlib.import_module(mod_name)
        obj = getattr(mod, name)
        if sec != section:
            lines += [f"## {sec}", ""]
            section = sec
        qual = f"{mod_name}.{name}"
        if inspect.isclass(obj):
            values = _enum_values(obj) if sec == "Events" else []
            header = f"### class `{name}`" if not values else f"### `{name}`"
            lines += [header, "", f"`{qual}`", ""]
            if not values:
                ctor = _ctor(obj)
                if ctor:
                    lines += [f"Constructor: `{name}{ctor}`", ""]
            doc = _doc(obj)
            if doc:
                lines += [doc, ""]
            if values:
                lines += ["| name | value |", "|---|---|"]
                lines += [f"| `{k}` | `{v!r}` |" for k, v in values]
                lines.append("")
                continue
            members = _members(obj)
            if members:
                lines += ["| member | kind | description |", "|---|---|---|"]
                for kind, mname, attr, aliases in members:
                    sig = "" if kind == "property" else _sig(attr, drop_first=_takes_self(attr))
                    desc = _doc(attr, first_paragraph=True).replace("\n", " ").replace("|", "\\|")
                    if aliases:
                        desc += " " * bool(desc) + "Alias: " + ", ".join(f"`{a}`" for a in aliases) + "."
                    lines.append(f"| `{mname}{sig}` | {kind} | {desc} |")
                lines.append("")
        else:
            lines += [f"### `{name}{_sig(obj)}`", "", f"`{qual}`", ""]
            doc = _doc(obj)
            if doc:
                lines += [doc, ""]
    return "\n".join(lines).rstrip() + "\n"


def main() -> int:
    text = render()
    if "--check" in sys.argv:
        current = OUT.read_text() if OUT.exists() else ""
        if current != text:
            print(f"{OUT} is stale: run python tools/gen_api_docs.py", file=sys.stderr)
            return 1
        return 0
    OUT.write_text(text)
    print(f"wrote {OUT} ({len(text.splitlines())} lines)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
