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
        self._label_fast()

    def _label_fast(self) -> None:
        """Every indexer a single-label index (the Pod cache's job-name index): upsert compares
        the label values of the old and new version and leaves the index alone when they are
        equal — a status update of a pod never touches it (measured: index upkeep was ~5 % of
        a shard worker's CPU, profiles/r2_pprof_v11_fused)."""
        labels = [(name, getattr(fn, "label", None)) for name, fn in self._indexers.items()]
        self._labels = labels if labels and all(lb for _, lb in labels) else None

    def add_indexer(self, name: str, fn: IndexFunc) -> None:
        self._indexers[name] = fn
        idx = self._indices[name] = {}
        for k, obj in self._items.items():
            for v in fn(obj):
                idx.setdefault(v, set()).add(k)
        self._label_fast()

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
        m = obj.get("metadata") or _EMPTY
        ns = m.get("namespace")
        key = f"{ns}/{m.get('name', '')}" if ns else m.get("name", "")  # kube.object_key, inlined
        items = self._items
        old = items.get(key)
        items[key] = obj
        labels = self._labels
        if labels is not None:
            new_l = m.get("labels") or _EMPTY
            old_l = ((old.get("metadata") or _EMPTY).get("labels") or _EMPTY) if old is not None else None
            indices = self._indices
            for name, label in labels:
                v = new_l.get(label)
                ov = old_l.get(label) if old_l is not None else None
                if v == ov:
                    continue
                idx = indices[name]
                if ov:
                    st = idx.get(ov)
                    if st is not None:
                        st.discard(key)
                        if not st:
                            del idx[ov]
                if v:
                    st = idx.get(v)
                    if st is None:
                        idx[v] = {key}
                    else:
                        st.add(key)
        elif self._indexers:
            if old is not None:
                self._unindex(key, old)
            self._index(key, obj)
        return old

    def delete(self, obj_or_key) -> Optional[Dict[str, Any]]:
        key = obj_or_key if isinstance(obj_or_key, str) else kube.object_key(obj_or_key)
        old = self._items.pop(key, None)
        if old is None or not self._indexers:
            return old
        labels = self._labels
        if labels is None:
            self._unindex(key, old)
            return old
        old_l = (old.get("metadata") or _EMPTY).get("labels") or _EMPTY
        for name, label in labels:
            v = old_l.get(label)
            if v:
                idx = self._indices[name]
                st = idx.get(v)
                if st is not None:
                    st.discard(key)
                    if not st:
                        del idx[v]
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

    fn.label = label  # type: ignore[attr-defined]  # lets Indexer take the label fast path
    return fn


_EMPTY: Dict[str, Any] = {}
