"""TEST INFRASTRUCTURE ONLY — CPU oracles for the vits_amd hot path.

Nothing under ``vits_amd/`` imports this package.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it,
and only as the checker / the timed CPU baseline, never as the product path.

* ``mas``          — C restatement of monotonic_align.maximum_path
                     (oracle/mas_oracle.c), ctypes-loaded.
* ``vits_oracle``  — functional torch-CPU fp32 restatement of the reference
                     forward/inference path (emotional-vits models.py,
                     modules.py, attentions.py, commons.py), driven by a plain
                     state_dict.
* ``stft_oracle``  — numpy/torch-CPU restatement of the STFT-loss and mel ops.
"""
