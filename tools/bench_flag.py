"""bench.py with one package module flag set (in-process A/B of a module-level choice):
    python tools/bench_flag.py real_motion_model._STACK_BF16_WEIGHTS=0 -- --dtype bf16 --no-trace
Only for runs without the nested trace child (--no-trace), which would not inherit the flag."""
import importlib
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
i = sys.argv.index('--')
for spec in sys.argv[1:i]:
    name, val = spec.split('=')
    mod, attr = name.rsplit('.', 1)
    m = importlib.import_module('a2m.' + mod)
    assert hasattr(m, attr), spec
    setattr(m, attr, type(getattr(m, attr))(int(val)))
sys.argv = [os.path.join(REPO, 'bench.py')] + sys.argv[i + 1:]
assert '--no-trace' in sys.argv
runpy.run_path(sys.argv[0], run_name='__main__')
