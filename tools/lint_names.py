#!/usr/bin/env python3
"""Cheap undefined-global-name check (pyflakes is not installed): reports names loaded in a module that are never
bound anywhere in it (imports, defs, assignments, args, comprehension targets) nor builtins. Catches the class of
bug where a module-level table is deleted by an edit but a GPU-only path still uses it (CPU tests cannot see it)."""
import ast
import builtins
import pathlib
import sys


def undefined(path):
    tree = ast.parse(pathlib.Path(path).read_text())
    bound = set(dir(builtins)) | {"__file__", "__name__", "__doc__"}
    for n in ast.walk(tree):
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            bound.add(n.name)
        elif isinstance(n, ast.Import):
            bound.update((a.asname or a.name).split(".")[0] for a in n.names)
        elif isinstance(n, ast.ImportFrom):
            bound.update(a.asname or a.name for a in n.names)
        elif isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            bound.add(n.id)
        elif isinstance(n, ast.arg):
            bound.add(n.arg)
        elif isinstance(n, ast.ExceptHandler) and n.name:
            bound.add(n.name)
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            bound.update(n.names)
    star = any(isinstance(n, ast.ImportFrom) and any(a.name == "*" for a in n.names) for n in ast.walk(tree))
    if star:
        return []
    used = {(n.id, n.lineno) for n in ast.walk(tree) if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load)}
    return sorted((ln, nm) for nm, ln in used if nm not in bound)


def main(roots):
    bad = 0
    for r in roots:
        for p in sorted(pathlib.Path(r).rglob("*.py")):
            for ln, nm in undefined(p):
                print(f"{p}:{ln}: undefined name {nm!r}")
                bad += 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or ["deeplearning4j_amd"]))
