"""JavaScript value semantics needed for line-by-line parity with the reference.

Python and JavaScript disagree on truthiness: ``{}`` and ``[]`` are falsy in Python but
truthy in JS, so a guard like ``if (!p2pConfig ...)`` (``lib/hlsjs-p2p-wrapper-private.js:128``)
must not be ported as ``if not p2pConfig``.
"""
from __future__ import annotations

import math
from typing import Any


def truthy(v: Any) -> bool:
    """``Boolean(v)`` in JavaScript: false only for undefined/null, false, 0/-0/NaN and ''."""
    if v is None or v is False:
        return False
    if isinstance(v, bool):
        return True
    if isinstance(v, (int, float)):
        return not (v == 0 or (isinstance(v, float) and math.isnan(v)))
    if isinstance(v, str):
        return v != ""
    return True  # objects, arrays, functions — including empty ones
