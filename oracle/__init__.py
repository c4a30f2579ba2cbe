"""CPU oracle for the tri-modal residual-attention hot path -- TEST INFRASTRUCTURE ONLY.

This package is a from-scratch, functional restatement (PyTorch fp32 on the CPU) of the
reference's model, loss and train-step arithmetic.  It is the *checker*: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.  The
product path (``multimodal-emotion-processing_amd``) never imports, links or falls back to it.

Pinning: the restatement is validated against golden vectors produced by the reference's own
classes (AST-extracted from ``/root/reference``; see ``tests/golden/make_golden.py``) and the
fixtures are committed under ``tests/golden/``.  The reference itself ships no tests, fixtures
or known-answer vectors, so those generated fixtures are the only pin.

Modules:
  common      attention core, LayerNorm, circle loss, clip-norm, AdamW / Adam (torch semantics)
  cmu_mosei   ``Concat_Trans`` / ``Multi_ATTN`` family      (cmu-mosei/run.py:206-390)
  realformer  ``State_Transfer`` / ``Multi_class`` family  (others/realformer.py:133-335)
  ren_mme     ``Base_model`` family + R-Drop KL loss       (Ren-MME/run.py:157-340)
"""
