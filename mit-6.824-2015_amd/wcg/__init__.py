"""wcg - MI355X-native word count for the Lab 1 MapReduce hot path of wushan270/mit-6.824-2015.

Python host side (tests, bench, multi-GPU orchestration) over the C ABI of libwcg.so
(include/wcg.h).  The compute path is hand-written HIP for gfx950; there is no CPU fallback.
"""
from ._lib import (Engine, WcgError, ihash, load, version, EXPORTED, RECORD_BYTES,  # noqa: F401
                   exchange_plan, gather_plan, exchange_local, gather_merge_local)
