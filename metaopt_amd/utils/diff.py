"""Colored unified diff (reference: ``src/orion/core/utils/diff.py:15-46``)."""
from __future__ import annotations

import difflib

RED, GREEN, BLUE, END = "\033[31m", "\033[32m", "\033[34m", "\033[0m"


def colored_diff(a: str, b: str) -> str:
    lines = []
    for line in difflib.unified_diff(a.splitlines(), b.splitlines(), lineterm=""):
        if line.startswith(("+++", "---")):
            lines.append(line)
        elif line.startswith("+"):
            lines.append(GREEN + line + END)
        elif line.startswith("-"):
            lines.append(RED + line + END)
        elif line.startswith("@@"):
            lines.append(BLUE + line + END)
        else:
            lines.append(line)
    return "\n".join(lines)
