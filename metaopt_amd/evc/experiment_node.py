"""Experiment nodes of the version-control tree and tree-wide trial fetching
(reference: ``src/orion/core/evc/experiment.py:28-225``).

Nodes load lazily from storage: the parent from ``refers.parent_id``, the children by querying
``refers.parent_id == this id``.  ``fetch_trials`` returns this experiment's trials plus every
ancestor's trials adapted *forward* through each branch's adapter, and every descendant's trials
adapted *backward* -- all expressed in this experiment's space.
"""
from __future__ import annotations

from typing import List

from .tree import TreeNode


class ExperimentNode(TreeNode):
    __slots__ = ("name", "version", "_no_parent_lookup", "_no_children_lookup", "_storage")

    def __init__(self, name, version, experiment=None, parent=None, children=(), storage=None):
        super().__init__(experiment, parent, children)
        self.name = name
        self.version = version
        self._no_parent_lookup = True
        self._no_children_lookup = True
        self._storage = storage

    def _get_storage(self):
        if self._storage is not None:
            return self._storage
        from ..storage.protocol import get_storage
        return get_storage()

    @property
    def item(self):
        if self._item is None:
            from ..core.experiment import ExperimentView
            self._item = ExperimentView(self.name, version=self.version,
                                        storage=self._get_storage())
            self._item.connect_to_version_control_tree(self)
        return self._item

    @item.setter
    def item(self, value):
        self._item = value

    @property
    def parent(self):
        if self._parent is None and self._no_parent_lookup:
            self._no_parent_lookup = False
            pid = self.item.refers.get("parent_id")
            if pid is not None:
                found = self._get_storage().fetch_experiments({"_id": pid},
                                                              {"name": 1, "version": 1})
                if found:
                    p = found[0]
                    node = ExperimentNode(p["name"], p.get("version", 1), storage=self._storage)
                    self.set_parent(node)
                    node._no_children_lookup = True
        return self._parent

    @property
    def children(self):
        if self._no_children_lookup:
            self._no_children_lookup = False
            existing = list(self._children)
            found = self._get_storage().fetch_experiments({"refers.parent_id": self.item.id},
                                                          {"name": 1, "version": 1})
            for c in found:
                if any(e.name == c["name"] and e.version == c.get("version", 1)
                       for e in existing):
                    continue
                child = ExperimentNode(c["name"], c.get("version", 1), storage=self._storage)
                child._no_parent_lookup = False
                self.add_children(child)
        return self._children

    @property
    def adapter(self):
        return self.item.refers["adapter"]

    @property
    def tree_name(self):
        return f"{self.name}-v{self.item.version}"

    # -- tree-wide trial fetching ----------------------------------------------------------------
    def fetch_trials(self):
        return self._fetch_trials("fetch_trials")

    def fetch_pending_trials(self):
        return self._fetch_trials("fetch_pending_trials")

    def fetch_noncompleted_trials(self):
        return self._fetch_trials("fetch_noncompleted_trials")

    def fetch_trials_by_status(self, status):
        return self._fetch_trials("fetch_trials_by_status", status)

    def fetch_lost_trials(self):
        return self._fetch_trials("fetch_lost_trials")

    def _own(self, node, fun_name, args):
        exp = node.item
        fn = getattr(exp, fun_name, None)
        if fn is not None:
            try:
                return list(fn(*args, with_evc_tree=False))
            except TypeError:
                return list(fn(*args))
        return list(getattr(exp.storage, fun_name)(exp, *args))

    def _fetch_trials(self, fun_name, *args) -> List:
        trials = self._own(self, fun_name, args)
        # ancestors: adapt forward along the chain down to this node
        chain = []
        node = self
        while node.parent is not None:
            chain.append(node)
            node = node.parent
            parent_trials = self._own(node, fun_name, args)
            for child in reversed(chain):
                parent_trials = child.adapter.forward(parent_trials)
            trials += parent_trials
        # descendants: adapt backward up to this node

        def rec(n, path):
            nonlocal trials
            for c in n.children:
                t = self._own(c, fun_name, args)
                for a in [c] + path[::-1]:
                    t = a.adapter.backward(t)
                trials += t
                rec(c, path + [c])

        rec(self, [])
        return trials
