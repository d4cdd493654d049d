#!/usr/bin/env python3
"""AsyncEA client role (reference: examples/EASGD_client.lua); see examples/easgd.py."""
import os
import runpy
import sys

sys.argv = [sys.argv[0], "--role", "client"] + sys.argv[1:]
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "easgd.py"), run_name="__main__")
