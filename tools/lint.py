#!/usr/bin/env python3
"""Static checks for the Python sources (the reference's ``npm run lint`` = eslint over ``lib/``
and ``test/``, ``package.json:22``; no Python linter ships in this image, so the checks that
matter here are implemented on the ``ast`` module):

    L001  unused module-level import (``__init__.py`` re-exports and ``__all__`` count as used)
    L002  bare ``except:``
    L003  mutable default argument (list / dict / set literal or constructor call)
    L004  ``is`` / ``is not`` against a str / bytes / number literal
    L005  f-string without placeholders
    L006  name redefined in the same class / module body before any use (shadowed def)
    L007  tab indentation or trailing whitespace
    L008  line longer than 120 characters
    L009  ``assert`` on a non-empty tuple (always true)

A line carrying ``# noqa`` is exempt.  Exit status 1 when anything is reported.

    python tools/lint.py                  # package, tests, tools, examples, bench.py, setup.py
    python tools/lint.py path/to/file.py  # selected files / directories
"""
from __future__ import annotations

import ast
import sys
from pathlib import Path
from typing import Iterable, List, Tuple

REPO = Path(__file__).resolve().parents[1]
DEFAULT_TARGETS = ["hlsjs_p2p_wrapper_amd", "tests", "tools", "examples", "bench.py", "setup.py", "__graft_entry__.py"]
MAX_LINE = 120
Finding = Tuple[str, int, str, str]  # path, line, code, message


def _py_files(targets: Iterable[str]) -> List[Path]:
    out: List[Path] = []
    for t in targets:
        p = (REPO / t) if not Path(t).is_absolute() else Path(t)
        if p.is_dir():
            out.extend(sorted(q for q in p.rglob("*.py") if "build" not in q.parts and "__pycache__" not in q.parts))
        elif p.suffix == ".py" and p.exists():
            out.append(p)
    return out


def _names_used(tree: ast.AST) -> set:
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            root = node
            while isinstance(root, ast.Attribute):
                root = root.value
            if isinstance(root, ast.Name):
                used.add(root.id)
    # names inside string annotations ("Optional[SwarmNode]") and __all__ entries (docstrings
    # and other strings do not count)
    strings = []
    for node in ast.walk(tree):
        if isinstance(node, ast.arg) and node.annotation is not None:
            strings.append(node.annotation)
        elif isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)) and node.returns is not None:
            strings.append(node.returns)
        elif isinstance(node, ast.AnnAssign):
            strings.append(node.annotation)
        elif isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            strings.append(node.value)
    for ann in strings:
        for c in ast.walk(ann):
            if isinstance(c, ast.Constant) and isinstance(c.value, str):
                used.update(_identifiers(c.value))
    return used


def _identifiers(text: str) -> Iterable[str]:
    word = []
    for ch in text + " ":
        if ch.isalnum() or ch == "_":
            word.append(ch)
        elif word:
            yield "".join(word)
            word = []


def _is_mutable_default(node: ast.AST) -> bool:
    if isinstance(node, (ast.List, ast.Dict, ast.Set, ast.ListComp, ast.DictComp, ast.SetComp)):
        return True
    return (isinstance(node, ast.Call) and isinstance(node.func, ast.Name)
            and node.func.id in ("list", "dict", "set", "bytearray"))


def _check_tree(path: Path, tree: ast.AST, lines: List[str]) -> List[Finding]:
    rel = str(path.relative_to(REPO)) if path.is_relative_to(REPO) else str(path)
    out: List[Finding] = []

    def add(node_or_line, code: str, msg: str) -> None:
        ln = node_or_line if isinstance(node_or_line, int) else node_or_line.lineno
        if 0 < ln <= len(lines) and "noqa" in lines[ln - 1]:
            return
        out.append((rel, ln, code, msg))

    # L001 unused imports (module level only; conditional imports inside try/if included)
    if path.name != "__init__.py":
        used = _names_used(tree)
        for node in tree.body if isinstance(tree, ast.Module) else []:
            for imp in _module_imports(node):
                if isinstance(imp, ast.ImportFrom) and imp.module == "__future__":
                    continue
                for alias in imp.names:
                    if alias.name == "*":
                        continue
                    bound = alias.asname or alias.name.split(".")[0]
                    if alias.asname and alias.asname == alias.name:  # `import x as x` = re-export
                        continue
                    if bound not in used:
                        add(imp, "L001", f"'{alias.name}' imported but unused")

    format_specs = {id(n.format_spec) for n in ast.walk(tree)
                    if isinstance(n, ast.FormattedValue) and n.format_spec is not None}
    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            add(node, "L002", "bare 'except:' (catch Exception or narrower)")
        elif isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
            for d in list(node.args.defaults) + [d for d in node.args.kw_defaults if d is not None]:
                if _is_mutable_default(d):
                    add(d, "L003", "mutable default argument")
        elif isinstance(node, ast.Compare):
            for op, right in zip(node.ops, node.comparators):
                if isinstance(op, (ast.Is, ast.IsNot)) and isinstance(right, ast.Constant) \
                        and isinstance(right.value, (str, bytes, int, float)) and not isinstance(right.value, bool):
                    add(node, "L004", "'is' comparison with a literal")
        elif isinstance(node, ast.JoinedStr) and id(node) not in format_specs:
            if not any(isinstance(v, ast.FormattedValue) for v in node.values):
                add(node, "L005", "f-string without placeholders")
        elif isinstance(node, ast.Assert):
            if isinstance(node.test, ast.Tuple) and node.test.elts:
                add(node, "L009", "assert on a tuple is always true")
        if isinstance(node, (ast.Module, ast.ClassDef)):
            _check_redefinitions(node, add)

    for i, line in enumerate(lines, 1):
        stripped = line.rstrip("\n")
        if stripped != stripped.rstrip():
            add(i, "L007", "trailing whitespace")
        if stripped[: len(stripped) - len(stripped.lstrip())].count("\t"):
            add(i, "L007", "tab indentation")
        if len(stripped) > MAX_LINE:
            add(i, "L008", f"line too long ({len(stripped)} > {MAX_LINE})")
    return out


def _module_imports(node: ast.AST):
    if isinstance(node, (ast.Import, ast.ImportFrom)):
        yield node
    elif isinstance(node, ast.Try):
        for sub in node.body + node.orelse + node.finalbody + [s for h in node.handlers for s in h.body]:
            yield from _module_imports(sub)
    elif isinstance(node, ast.If):
        for sub in node.body + node.orelse:
            yield from _module_imports(sub)


def _check_redefinitions(scope: ast.AST, add) -> None:
    """A def / class bound twice in one body with no use of the name in between (the first
    binding is dead).  Property setters (``@x.setter``) and ``typing.overload`` are fine."""
    defined = {}
    for stmt in scope.body:
        if isinstance(stmt, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            decos = getattr(stmt, "decorator_list", [])
            is_accessor = any(isinstance(d, ast.Attribute) and d.attr in ("setter", "getter", "deleter")
                              for d in decos)
            is_overload = any((isinstance(d, ast.Name) and d.id == "overload")
                              or (isinstance(d, ast.Attribute) and d.attr == "overload") for d in decos)
            if stmt.name in defined and not is_accessor and not is_overload:
                add(stmt, "L006", f"redefinition of '{stmt.name}' from line {defined[stmt.name]}")
            defined[stmt.name] = stmt.lineno
        else:
            # any reference to a name in between makes the earlier binding live
            for n in ast.walk(stmt):
                if isinstance(n, ast.Name) and n.id in defined:
                    del defined[n.id]


def lint(paths: Iterable[Path]) -> List[Finding]:
    findings: List[Finding] = []
    for path in paths:
        src = path.read_text()
        try:
            tree = ast.parse(src, filename=str(path))
        except SyntaxError as e:
            findings.append((str(path), e.lineno or 0, "E999", f"syntax error: {e.msg}"))
            continue
        findings.extend(_check_tree(path, tree, src.splitlines()))
    return findings


def main(argv: List[str]) -> int:
    files = _py_files(argv or DEFAULT_TARGETS)
    findings = lint(files)
    for rel, ln, code, msg in findings:
        print(f"{rel}:{ln}: {code} {msg}")
    print(f"{len(files)} files, {len(findings)} findings", file=sys.stderr)
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
