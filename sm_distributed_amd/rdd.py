"""A minimal in-process stand-in for the pyspark RDD surface the hot path's callers use.

The reference passes Spark RDDs between compute_sf_images, sf_image_metrics, filter_sf_images and
SearchResults (search_algorithm.py:24-25, search_results.py:110).  There is no Spark in the GPU path:
this class offers the same method names (map / flatMap / filter / mapValues / collect / take / count /
foreachPartition / keys / values / first) over a local list so those callers keep working.
"""
from __future__ import annotations


class LocalRDD:
    def __init__(self, items):
        self._items = list(items)

    # transformations
    def map(self, f):
        return LocalRDD(f(x) for x in self._items)

    def flatMap(self, f):
        return LocalRDD(y for x in self._items for y in f(x))

    def filter(self, f):
        return LocalRDD(x for x in self._items if f(x))

    def mapValues(self, f):
        return LocalRDD((k, f(v)) for k, v in self._items)

    def keys(self):
        return LocalRDD(k for k, _ in self._items)

    def values(self):
        return LocalRDD(v for _, v in self._items)

    def cache(self):
        return self

    persist = cache

    def coalesce(self, *_a, **_k):
        return self

    # actions
    def collect(self):
        return list(self._items)

    def take(self, n):
        return list(self._items[:n])

    def first(self):
        return self._items[0]

    def count(self):
        return len(self._items)

    def foreach(self, f):
        for x in self._items:
            f(x)

    def foreachPartition(self, f):
        f(iter(self._items))

    def __iter__(self):
        return iter(self._items)

    def __len__(self):
        return len(self._items)


def parallelize(items, *_a, **_k):
    """``sc.parallelize`` equivalent for tests and local callers."""
    return LocalRDD(items)
