"""CPU oracle for the PoSFeat extraction + correlation hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``posfeat_amd/`` imports this package:
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may use it, and only as the checker / the timed CPU baseline.

Contents (each function cites the reference file:line it restates):

* ``model_ref``   -- torch-CPU fp32 restatement of ResUNet (with the
  torchvision ResNet-50 encoder restated from its published architecture,
  torchvision being absent here), KeypointDet and ``PoSFeat.extract``.
* ``detect_ref``  -- numpy restatement of ``generate_kpts_single`` / ``nms`` /
  ``sample_feat_by_coord`` / coordinate (de)normalisation, with the stated
  tie rule.

Pinning: the restatement is checked against golden vectors produced by
running the reference's own Python (``/root/reference``) in the build
container -- see ``tests/golden/gen_golden.py`` and
``tests/test_oracle_golden.py``.
"""
