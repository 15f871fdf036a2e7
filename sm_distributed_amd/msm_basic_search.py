"""Alias module matching the reference layout (sm/engine/msm_basic/msm_basic_search.py)."""
from .search_algorithm import MSMBasicSearch, SearchAlgorithm  # noqa: F401
