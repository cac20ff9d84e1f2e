"""Logging configuration.

The reference logs with ``console.warn`` / ``console.error`` (retries, final failures,
engine errors, unparsed levels) and strips ALL console output from production builds
(uglify ``drop_console``, ``Gruntfile.js:26``); debug verbosity is driven by
``p2pConfig.debug`` (agent) and ``hlsjsConfig.debug`` (engine).

Here every module logs to a child of the ``hlsjs_p2p_wrapper_amd`` logger:

* production (``HLSJS_P2P_ENV=production`` at build or run time) -> the package logger
  drops everything (the ``drop_console`` analog);
* ``configure(debug=True)`` (``p2pConfig.debug`` / ``hlsjsConfig.debug``) -> DEBUG level
  with a stderr handler; otherwise WARNING and above reach the root handlers.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

ROOT = "hlsjs_p2p_wrapper_amd"
_handler: Optional[logging.Handler] = None


def environment() -> str:
    env = os.environ.get("HLSJS_P2P_ENV")
    if env:
        return env
    try:
        from .. import _build_info  # written by setup.py

        return getattr(_build_info, "ENVIRONMENT", "development")
    except ImportError:
        return "development"


def configure(debug: Optional[bool] = None) -> logging.Logger:
    global _handler
    log = logging.getLogger(ROOT)
    if environment() == "production":
        log.handlers[:] = [logging.NullHandler()]
        log.propagate = False
        log.setLevel(logging.CRITICAL + 1)
        return log
    if debug:
        if _handler is None:
            _handler = logging.StreamHandler()
            _handler.setFormatter(logging.Formatter("[%(name)s] %(levelname)s %(message)s"))
            log.addHandler(_handler)
        log.setLevel(logging.DEBUG)
    elif debug is not None and log.level == logging.DEBUG:
        log.setLevel(logging.WARNING)
    return log
