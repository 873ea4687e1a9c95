"""Oracle host-side logic: windowing, decision rule, smoothing/aggregation, JSON.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates ``inference_runner.py:176-190`` (slice_waveform),
``:194-214`` (interpret_multihead_logits) and ``:300-353`` (smoothing,
percentages, segments, JSON dict).  Pinned by the fixtures generated from the
reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch


def slice_waveform(wf: torch.Tensor, sr: int, cfg):
    """inference_runner.py:176-190."""
    window_samples = int(cfg.window_size * sr)
    hop_samples = int((1 - cfg.overlap) * window_samples)
    chunks, timestamps = [], []
    for start_idx in range(0, wf.shape[0] - window_samples + 1, hop_samples):
        piece = wf[start_idx:start_idx + window_samples]
        if piece.abs().max() < cfg.silence_threshold:
            continue
        chunks.append(piece)
        timestamps.append(start_idx / sr)
    return chunks, timestamps


def interpret_multihead_logits(logits: torch.Tensor, threshold=0.5,
                               synthetic_names: List[str] = None, real_name: str = 'Real'):
    """inference_runner.py:194-214."""
    s = torch.sigmoid(logits)
    n = s.shape[0] - 1
    syn_probs = s[:n]
    real_prob = s[-1]
    if real_prob >= threshold and (syn_probs < threshold).all():
        label = real_name
    else:
        idx = int(torch.argmax(syn_probs).item())
        if synthetic_names and idx < len(synthetic_names):
            label = synthetic_names[idx]
        else:
            label = f'Synthetic_{idx + 1}'
    return label, s.cpu().numpy()


def aggregate(filename, outputs: torch.Tensor, timestamps, threshold, synthetic_names, real_name,
              smooth=False, window_size=4.0):
    """inference_runner.py:292-349 -> the JSON dict."""
    from scipy.ndimage import gaussian_filter1d
    raw_labels, raw_probs = [], []
    for row in outputs:
        label, s = interpret_multihead_logits(row, threshold, synthetic_names, real_name)
        raw_labels.append(label)
        raw_probs.append(s)
    if smooth:
        arr = np.array(raw_probs)
        for dim in range(arr.shape[1]):
            arr[:, dim] = gaussian_filter1d(arr[:, dim], sigma=2)
        for i in range(arr.shape[0]):
            row_sum = arr[i].sum()
            if row_sum > 0:
                arr[i] /= row_sum
        labels2 = []
        for i in range(arr.shape[0]):
            real_p = arr[i, -1]
            syn_p = arr[i, :-1]
            if real_p >= threshold and (syn_p < threshold).all():
                labels2.append(real_name)
            else:
                idx = int(syn_p.argmax())
                labels2.append(synthetic_names[idx] if idx < len(synthetic_names) else f'Synthetic_{idx + 1}')
        raw_labels = labels2
        raw_probs = arr.tolist()
    final = np.mean(raw_probs, axis=0)
    prob = {}
    n_syn = len(final) - 1
    for i in range(n_syn):
        name = synthetic_names[i] if i < len(synthetic_names) else f'Synthetic_{i + 1}'
        prob[name] = float(final[i] * 100)
    prob[real_name] = float(final[-1] * 100)
    segments = [{'start_sec': timestamps[i], 'end_sec': timestamps[i] + window_size, 'label': lbl}
                for i, lbl in enumerate(raw_labels)]
    return {'filename': filename, 'segments': segments, 'percentages': prob}
