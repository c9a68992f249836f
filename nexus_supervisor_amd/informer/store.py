"""Thread-unsafe (loop-confined) object cache with secondary indexes — the
client-go ``cache.Indexer`` equivalent used by the informers."""
from __future__ import annotations

from typing import Any, Callable, Dict, Iterable, List, Optional, Set

from ..models import kube

IndexFunc = Callable[[Dict[str, Any]], Iterable[str]]


class Indexer:
    def __init__(self, indexers: Optional[Dict[str, IndexFunc]] = None):
        self._items: Dict[str, Dict[str, Any]] = {}
        self._indexers: Dict[str, IndexFunc] = dict(indexers or {})
        self._indices: Dict[str, Dict[str, Set[str]]] = {n: {} for n in self._indexers}

    def add_indexer(self, name: str, fn: IndexFunc) -> None:
        self._indexers[name] = fn
        idx = self._indices[name] = {}
        for k, obj in self._items.items():
            for v in fn(obj):
                idx.setdefault(v, set()).add(k)

    def _unindex(self, key: str, obj: Dict[str, Any]) -> None:
        for name, fn in self._indexers.items():
            idx = self._indices[name]
            for v in fn(obj):
                s = idx.get(v)
                if s is not None:
                    s.discard(key)
                    if not s:
                        del idx[v]

    def _index(self, key: str, obj: Dict[str, Any]) -> None:
        for name, fn in self._indexers.items():
            idx = self._indices[name]
            for v in fn(obj):
                idx.setdefault(v, set()).add(key)

    def upsert(self, obj: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        key = kube.object_key(obj)
        old = self._items.get(key)
        if old is not None and self._indexers:
            self._unindex(key, old)
        self._items[key] = obj
        if self._indexers:
            self._index(key, obj)
        return old

    def delete(self, obj_or_key) -> Optional[Dict[str, Any]]:
        key = obj_or_key if isinstance(obj_or_key, str) else kube.object_key(obj_or_key)
        old = self._items.pop(key, None)
        if old is not None and self._indexers:
            self._unindex(key, old)
        return old

    def get(self, key: str) -> Optional[Dict[str, Any]]:
        return self._items.get(key)

    def get_by_name(self, namespace: str, name: str) -> Optional[Dict[str, Any]]:
        return self._items.get(f"{namespace}/{name}" if namespace else name)

    def by_index(self, name: str, value: str) -> List[Dict[str, Any]]:
        keys = self._indices.get(name, {}).get(value, ())
        return [self._items[k] for k in keys if k in self._items]

    def replace(self, objs: Iterable[Dict[str, Any]]) -> Dict[str, Dict[str, Any]]:
        """Swap contents (re-list); returns the previous item map."""
        old = self._items
        self._items = {}
        self._indices = {n: {} for n in self._indexers}
        for o in objs:
            self.upsert(o)
        return old

    def keys(self):
        return list(self._items.keys())

    def values(self):
        return list(self._items.values())

    def __len__(self) -> int:
        return len(self._items)

    def __contains__(self, key) -> bool:
        return key in self._items


def label_index(label: str) -> IndexFunc:
    def fn(obj):
        v = kube.labels_of(obj).get(label)
        return (v,) if v else ()

    return fn
