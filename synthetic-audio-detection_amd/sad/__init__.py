"""sad -- MI355X-native synthetic-audio-detection hot path.

Host-side Python over the C-ABI HIP library ``libsad.so`` (csrc/).  The public
drop-in surface mirrors the reference's modules (``inference_runner``,
``model_merger``, ``submodel_trainer`` one directory up); this package holds the
plumbing: library loader, device plans, synthetic data and weights.
"""
