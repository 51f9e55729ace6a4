"""Select the dispatches of graph-replayed bench steps from rocprofv3 CSVs.

tools/step_pmc.py runs the eager warm-up and the capture, synchronises, launches one marker
kernel (torch.cuda._sleep -> a kernel whose name holds MARKER) and only then replays the step
graph R times.  Every dispatch after the last marker (by Dispatch_Id, which the runtime
assigns in submission order) is a replayed-step dispatch; first-call weight repacks, the eager
steps' copies and the capture's warm-up are all before it.
"""
import csv
import glob
import os

MARKERS = ('spin_kernel', 'sleep')


def _did(row):
    for k in ('Dispatch_Id', 'Correlation_Id'):
        if row.get(k):
            return int(row[k])
    raise KeyError('no Dispatch_Id / Correlation_Id column')


def is_marker(name):
    n = name.lower()
    return any(m in n for m in MARKERS) and 'a2m' not in n


def replayed(rows):
    """rows (dicts with Kernel_Name and Dispatch_Id) after the last marker dispatch."""
    marks = [_did(r) for r in rows if is_marker(r.get('Kernel_Name', ''))]
    if not marks:
        raise SystemExit('replay_filter: no marker dispatch found (is this a tools/step_pmc.py run?)')
    cut = max(marks)
    return [r for r in rows if _did(r) > cut]


def load(d, pattern):
    files = glob.glob(os.path.join(d, '**', pattern), recursive=True) if os.path.isdir(d) else [d]
    if not files:
        raise SystemExit(f'no {pattern} under {d}')
    rows = []
    for fn in files:
        with open(fn, newline='') as f:
            rows.extend(csv.DictReader(f))
    return rows
