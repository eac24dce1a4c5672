#!/usr/bin/env python3
"""Profiling-only: run a script (argv[1], with the rest as its argv) with faulthandler dumping every thread's
Python stack to stderr every FH_SECONDS (default 240) -- to see where a long silent multi-rank run is."""
import faulthandler
import os
import runpy
import sys

faulthandler.dump_traceback_later(int(os.environ.get("FH_SECONDS", "240")), repeat=True, file=sys.stderr)
script = sys.argv[1]
sys.argv = sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
runpy.run_path(script, run_name="__main__")
