"""Config-code fingerprint used to guard resume.

The reference hashes ``dill.dumps`` of a position-stripped AST
(experiment-runner/__main__.py:27-49).  That digest depends on the interpreter
and dill versions (SURVEY §2.2 row 2 measured a different value on Py 3.10),
so a resume on another machine always trips the md5 prompt.

``ast_md5`` hashes ``ast.dump(tree, include_attributes=False)`` with every
docstring blanked: comments, blank lines, positions and docstrings do not
change it, and it is stable across CPython versions that share the AST node
set.  ``legacy_md5`` reproduces the reference scheme for reading old
``metadata.json`` files; ``matches`` accepts either.
"""
from __future__ import annotations

import ast
import hashlib
from typing import Optional

from .models import Metadata


def _strip_docstrings(tree: ast.AST) -> ast.AST:
    for node in ast.walk(tree):
        if isinstance(node, (ast.Module, ast.ClassDef, ast.FunctionDef, ast.AsyncFunctionDef)):
            body = getattr(node, "body", None)
            if body and isinstance(body[0], ast.Expr) and isinstance(getattr(body[0], "value", None), ast.Constant) \
                    and isinstance(body[0].value.value, str):
                body[0].value.value = ""
    return tree


def ast_md5(source: str, filename: str = "<config>") -> bytes:
    tree = ast.parse(source, filename=filename)
    _strip_docstrings(tree)
    return hashlib.md5(ast.dump(tree, include_attributes=False).encode("utf-8")).digest()


def legacy_md5(source: str, filename: str = "<config>") -> Optional[bytes]:
    """Reference-compatible digest (dill pickle of the zero-positioned AST).
    Returns None when dill is unavailable."""
    try:
        import dill  # noqa: F401
    except Exception:  # pragma: no cover
        return None
    tree = compile(source, filename, "exec", flags=ast.PyCF_ONLY_AST, optimize=0)
    for node in ast.walk(tree):
        for attr in ("lineno", "col_offset", "end_lineno", "end_col_offset"):
            if hasattr(node, attr):
                setattr(node, attr, 0)
    _strip_docstrings(tree)
    return hashlib.md5(dill.dumps(tree)).digest()


def fingerprint(source: str, filename: str = "<config>") -> Metadata:
    return Metadata(ast_md5(source, filename), scheme="ast-v2")


def matches(stored: Metadata, source: str, filename: str = "<config>") -> bool:
    if stored.md5sum == ast_md5(source, filename):
        return True
    legacy = legacy_md5(source, filename)
    return legacy is not None and stored.md5sum == legacy
