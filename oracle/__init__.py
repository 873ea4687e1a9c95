"""CPU oracle for the mel -> ResNet-18 -> ensemble hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the package under
``synthetic-audio-detection_amd/``) may import this package; only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and
only as the checker / the timed CPU baseline.

What it is: a pure-torch fp32 restatement of the reference's algorithm
(TtesseractT/Synthetic-Audio-Detection @ 2025-05-23) for this path.  The
reference delegates its arithmetic to torchaudio / torchvision / timm, none of
which is installed here, so the glue those libraries add is restated from their
documented semantics on top of the same torch
primitives they call (``torch.stft``, ``F.interpolate``, ``F.conv2d``).

How it is pinned (see tests/golden/make_golden.py and DESIGN.md "Oracle"):
  * the reference's own pure-torch functions (slice_waveform,
    interpret_multihead_logits, ModularMultiHeadClassifier, load_merged_model,
    waveform_to_spectrogram's glue, model_merger's save format and main()'s
    JSON writer) were imported from /root/reference with stub third-party
    modules and run to produce the committed fixtures in tests/golden/;
  * the restated third-party arithmetic is cross-checked against independent
    float64 implementations (numpy.fft.rfft; transformers.audio_utils
    .mel_filter_bank; transformers' ResNetModel for the backbone topology).
The torchaudio/torchvision/timm numerics themselves are therefore pinned only
through those independent restatements ("parity partially unpinned at the
third-party boundary").
"""
