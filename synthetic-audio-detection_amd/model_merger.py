#!/usr/bin/env python3
"""Drop-in replacement for the reference's ``modular/source/model_merger.py``:
merge N trained binary sub-models into one multi-head checkpoint.

Same CLI (``--submodels-folder --csv-file --model-name --output-path``), same
CSV schema (``model_filename,synthetic_class,real_class``,
modular/model-merge-example.csv:1), same output format
``{'state_dict': {sub_models.<i>.base.*, sub_models.<i>.head.*},
'metadata': {'class_names': [syn_1..syn_N, real]}}`` (model_merger.py:154-159).

Reference semantics kept on purpose:
``load_sub_model`` (model_merger.py:46-59) loads the trainer checkpoint with
``strict=False`` into ``BinaryClassifier`` (keys ``base.*``/``head.*``); the
trainer's keys are unprefixed timm keys plus ``head.*``, so only the head
matches and every sub-model keeps the backbone it was constructed with.  In the
reference that is timm's ImageNet ``pretrained=True`` backbone (a network
download, unavailable offline); here it is the deterministic random-init
backbone of ``BinaryClassifier(init='random')``.  Either way all N backbones
are identical, which the device engine exploits (one backbone run).
"""
from __future__ import annotations

import argparse
import collections
import csv
import os
import sys

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from inference_runner import BinaryClassifier, ModularMultiHeadClassifier  # noqa: E402,F401


def force_separate_parameters(model):
    """model_merger.py:42-44 (host tensors are already separate copies)."""
    for k, v in model.state_dict().items():
        model._sd[k] = v.clone()


def load_sub_model(checkpoint_path, device, model_name='resnet18'):
    """model_merger.py:46-59: BinaryClassifier + strict=False load of ck['state_dict']."""
    model = BinaryClassifier(model_name=model_name)
    ck = torch.load(checkpoint_path, map_location='cpu', weights_only=True)
    sd_in = ck['state_dict']
    model.load_state_dict(sd_in, strict=False)
    force_separate_parameters(model)
    return model


def merged_real_class(real_names):
    """model_merger.py:136-143: the common value, else the most common one."""
    if len(set(real_names)) == 1:
        return real_names[0]
    counter = collections.Counter(real_names)
    name = counter.most_common(1)[0][0]
    print('Warning: Not all real_class values match in CSV; using the most common value:', name)
    return name


def merge(entries, submodels_folder, model_name='resnet18', device='cpu'):
    """CSV rows (dicts) -> (ModularMultiHeadClassifier, class_names)."""
    sub_models, synthetic_names, real_names = [], [], []
    for i, entry in enumerate(entries, start=1):
        model_path = os.path.join(submodels_folder, entry['model_filename'])
        print(f"Loading sub-model {i} from {model_path} with synthetic class '{entry['synthetic_class']}' "
              f"and real class '{entry['real_class']}'")
        sub_models.append(load_sub_model(model_path, device, model_name=model_name))
        synthetic_names.append(entry['synthetic_class'])
        real_names.append(entry['real_class'])
    merged = ModularMultiHeadClassifier(sub_models, device if str(device).startswith('cuda') else 'cuda')
    return merged, synthetic_names + [merged_real_class(real_names)]


def main(argv=None):
    parser = argparse.ArgumentParser(description='Merge sub-models into a multi-head classifier with a merged Real output.')
    parser.add_argument('--submodels-folder', type=str, required=True, help='Folder containing sub-model .pth files.')
    parser.add_argument('--csv-file', type=str, required=True,
                        help='CSV file with columns "model_filename", "synthetic_class", and "real_class".')
    parser.add_argument('--model-name', type=str, default='resnet18')
    parser.add_argument('--output-path', type=str, required=True)
    args = parser.parse_args(argv)

    with open(args.csv_file, newline='') as csvfile:
        entries = list(csv.DictReader(csvfile))
    if not entries:
        print('No submodels found in CSV file!')
        return None
    merged, final_class_names = merge(entries, args.submodels_folder, args.model_name)
    if torch.cuda.is_available():  # reference :148-151 dummy forward, on the device path
        out = merged.forward_maps(torch.zeros(2, 128, 251))
        print('Merged model output shape:', tuple(out.shape))
    torch.save({'state_dict': merged.state_dict(), 'metadata': {'class_names': final_class_names}}, args.output_path)
    print(f'Saved merged model with metadata => {args.output_path}')
    return final_class_names


if __name__ == '__main__':
    main()
