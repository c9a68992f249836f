"""Informers: list+watch caches with indexers and Add/Update/Delete dispatch."""
from .informer import (
    ADDED,
    BOOKMARK,
    DELETED,
    ERROR,
    MODIFIED,
    InformerFactory,
    ListWatch,
    QueueListWatch,
    SharedInformer,
    WatchGone,
)
from .store import Indexer, label_index

__all__ = ["ADDED", "BOOKMARK", "DELETED", "ERROR", "MODIFIED", "InformerFactory", "ListWatch",
           "QueueListWatch", "SharedInformer", "WatchGone", "Indexer", "label_index"]
