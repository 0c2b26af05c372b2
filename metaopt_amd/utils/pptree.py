"""Pretty-print a tree of nodes (used by ``mopt list``; reference vendors ``pptree``)."""
from __future__ import annotations


def format_tree(node, children_attr="children", name=lambda n: str(n)) -> str:
    """Horizontal tree: root on the first line, children indented with box-drawing branches."""
    lines = []

    def _rec(n, prefix, is_last, is_root):
        label = name(n)
        if is_root:
            lines.append(label)
            child_prefix = ""
        else:
            lines.append(prefix + ("└" if is_last else "├") + "──" + label)
            child_prefix = prefix + ("   " if is_last else "│  ")
        kids = list(getattr(n, children_attr) or [])
        for i, k in enumerate(kids):
            _rec(k, child_prefix, i == len(kids) - 1, False)

    _rec(node, "", True, True)
    return "\n".join(lines)


def print_tree(node, children_attr="children", name=lambda n: str(n)):
    print(format_tree(node, children_attr, name))
