"""CPU oracle for the audio->pose hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything from this package, and only as the checker / CPU baseline -- never as
the thing measured or shipped.  The product path (``a2m``) never imports it.

Contents
  mel.py              numpy float64 restatement of pose_video/mel_features.py
  pyg_restatement.py  restatement of PyTorch-Geometric GATConv / GraphConv default
                      semantics (PyG is absent from the image and unpinned by the
                      reference: GNN parity is "parity unpinned" against real PyG, and
                      pinned only against this restatement run inside the reference)
  model.py            functional torch-CPU fp32 restatement of SelfAttention_G /
                      SelfAttention_D forward + the training-step losses
  weights.py          deterministic (numpy PCG64, keyed by state_dict name) weights
  synth.py            deterministic synthetic 16 kHz audio / pose inputs
  make_fixtures.py    imports the REFERENCE in this container (with stubs for its broken
                      import chain) and writes tests/golden/*.npz

Pinning: every function here is checked against the golden vectors produced by
running the reference itself (tests/test_oracle_golden.py).
"""
