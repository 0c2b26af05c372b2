"""Generic tree used by the experiment version-control tree
(reference: ``src/orion/core/evc/tree.py:23-419``).

``TreeNode`` holds an ``item``, one parent and ordered children; iteration is pre-order
(``PreOrderTraversal``), ``DepthFirstTraversal`` yields leaves first.  ``map(fn)`` builds a new
tree of the same shape with ``fn(node)`` as items.
"""
from __future__ import annotations


class PreOrderTraversal:
    def __init__(self, tree_node):
        self.stack = [tree_node]

    def __iter__(self):
        return self

    def __next__(self):
        if not self.stack:
            raise StopIteration
        node = self.stack.pop()
        self.stack.extend(reversed(list(node.children)))
        return node


class DepthFirstTraversal:
    """Post-order: every node after all of its descendants."""

    def __init__(self, tree_node):
        out = []

        def rec(n):
            for c in n.children:
                rec(c)
            out.append(n)

        rec(tree_node)
        self._it = iter(out)

    def __iter__(self):
        return self

    def __next__(self):
        return next(self._it)


class TreeNode:
    __slots__ = ("_item", "_parent", "_children")

    def __init__(self, item, parent=None, children=()):
        self._item = item
        self._parent = None
        self._children = []
        if parent is not None:
            self.set_parent(parent)
        self.add_children(*children)

    @property
    def item(self):
        return self._item

    @item.setter
    def item(self, value):
        self._item = value

    @property
    def parent(self):
        return self._parent

    def drop_parent(self):
        if self._parent is not None:
            self._parent._children = [c for c in self._parent._children if c is not self]
        self._parent = None

    def set_parent(self, node):
        if node is self._parent:
            return
        self.drop_parent()
        if node is not None:
            node._children.append(self)
        self._parent = node

    @property
    def children(self):
        return self._children

    def drop_children(self, *nodes):
        nodes = nodes or tuple(self._children)
        for n in nodes:
            if n in self._children:
                self._children = [c for c in self._children if c is not n]
                n._parent = None

    def add_children(self, *nodes):
        for n in nodes:
            if not isinstance(n, TreeNode):
                raise TypeError(f"Cannot add {type(n)} as a child: not a TreeNode")
            n.set_parent(self)

    @property
    def root(self):
        node = self
        while node.parent is not None:
            node = node.parent
        return node

    def map(self, function):
        """New tree (same shape, from self downwards) with items ``function(node)``."""
        new = TreeNode(function(self))
        for c in self.children:
            new.add_children(c.map(function))
        return new

    def __iter__(self):
        return PreOrderTraversal(self)

    def __repr__(self):
        return f"TreeNode({self.item})"


def flattened(trials_tree):
    """All trials of a tree of ``{'trials': [...]}`` items, pre-order."""
    return sum((node.item["trials"] for node in trials_tree), [])
