#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ (run from the repo root):

  python tests/golden/make_golden.py

1. reference_config.json — the literal hyper-parameters of the reference's config.py
   (rank/scaling_up/oneTrans/practice/config.py:9-117), read as TEXT with `ast` (no reference code
   is executed: TensorFlow is absent, and the file imports it at line 6).  Only needs
   /root/reference at generation time; the tests read the JSON.
2. c1_golden.npz / criteo_golden.npz — forward outputs, loss, per-bank gradient norms and gradient
   slices, and the parameters after one train step, computed by the float64 oracle
   (oracle/onetrans_ref.py) on seeded inputs, after checking it against the independent numpy
   restatement (oracle/onetrans_np.py) to 1e-12.  Parameters are regenerated from
   recommend_amd.params.init_params(seed) (Keras init, deterministic PCG64), so the fixture stays small.
"""

import ast
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, 'tests', 'golden')
REF_CONFIG = '/root/reference/rank/scaling_up/oneTrans/practice/config.py'


def extract_reference_config(path):
    tree = ast.parse(open(path).read())
    classes = {}
    for node in tree.body:
        if isinstance(node, ast.ClassDef):
            vals = {}
            for fn in node.body:
                if isinstance(fn, ast.FunctionDef) and fn.name == '__init__':
                    for st in fn.body:
                        if isinstance(st, ast.Assign) and len(st.targets) == 1:
                            t = st.targets[0]
                            if isinstance(t, ast.Attribute) and isinstance(t.value, ast.Name) and t.value.id == 'self':
                                try:
                                    vals[t.attr] = ast.literal_eval(st.value)
                                except ValueError:
                                    pass
            classes[node.name] = vals
    return classes


def small_criteo_cfg():
    from recommend_amd.config import workload_config
    cfg = workload_config('C2')
    cfg.hidden_dim, cfg.num_heads, cfg.ffn_dim, cfg.num_layers, cfg.num_ns_tokens = 32, 2, 64, 2, 3
    cfg.sparse_features = {k: 20 + i for i, k in enumerate(cfg.sparse_features)}
    cfg.seq_item_vocab = 50
    cfg._seq_lens = [4, 3, 5]
    return cfg


def c1_cfg():
    from recommend_amd.config import workload_config
    return workload_config('C1')


CASES = {
    'c1': (c1_cfg, 6),
    'criteo': (small_criteo_cfg, 5),
}


def make_case(name):
    import torch
    from recommend_amd.data import make_batch
    from recommend_amd.params import init_params, keras_variables
    from oracle import onetrans_np as N
    from oracle import onetrans_ref as R
    mk, B = CASES[name]
    cfg = mk()
    P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
    ns, seq, lab = make_batch(B, cfg, seed=1000)
    Pt = R.to_torch(P)
    out_l = R.forward(Pt, cfg, R.to_torch(ns), R.to_torch(seq), variant='literal')
    out_n = N.forward(P, cfg, ns, seq)
    for t in cfg.tasks:
        assert np.abs(out_l['logits'][t].numpy() - out_n['logits'][t]).max() < 1e-12
    loss, grads, out = R.loss_and_grads(Pt, cfg, R.to_torch(ns), R.to_torch(seq), R.to_torch(lab), training=True,
                                        seed=77, variant='literal')
    kv = keras_variables(cfg, {k: v.shape for k, v in P.items() if not k.startswith('emb.')})
    newP, _, loss2, _ = R.train_step(Pt, R.init_state(Pt, cfg), cfg, kv, R.to_torch(ns), R.to_torch(seq),
                                     R.to_torch(lab), seed=77, variant='literal')
    assert abs(float(loss) - float(loss2)) < 1e-12
    fx = {}
    for k, v in ns.items():
        fx[f'in.ns.{k}'] = v
    for k, v in seq.items():
        fx[f'in.seq.{k}'] = v
    for k, v in lab.items():
        fx[f'in.label.{k}'] = v
    for t in cfg.tasks:
        fx[f'out.logits.{t}'] = out_l['logits'][t].numpy()
        fx[f'out.probs.{t}'] = out_l['probs'][t].numpy()
        fx[f'train.logits.{t}'] = out['logits'][t].detach().numpy()
    fx['train.loss'] = np.array(float(loss))
    for k, g in grads.items():
        fx[f'grad.norm.{k}'] = np.array(float(torch.linalg.vector_norm(g)))
        fx[f'grad.head.{k}'] = g.reshape(-1)[:16].numpy()
    for k, w in newP.items():
        if not k.startswith('emb.'):
            fx[f'step1.head.{k}'] = w.detach().reshape(-1)[:16].numpy()
            fx[f'step1.norm.{k}'] = np.array(float(torch.linalg.vector_norm(w.detach())))
    np.savez_compressed(os.path.join(OUT, f'{name}_golden.npz'), **fx)
    print(f'{name}: {len(fx)} arrays, loss {float(loss):.10f}')


def main():
    if os.path.exists(REF_CONFIG):
        classes = extract_reference_config(REF_CONFIG)
        with open(os.path.join(OUT, 'reference_config.json'), 'w') as f:
            json.dump({'source': 'rank/scaling_up/oneTrans/practice/config.py (ast.literal_eval of __init__ '
                                 'assignments; not executed)', 'classes': classes}, f, indent=1, sort_keys=True)
        print('reference_config.json:', {k: len(v) for k, v in classes.items()})
    for name in CASES:
        make_case(name)


if __name__ == '__main__':
    main()
