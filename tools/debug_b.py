import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from test_model_gpu import small_criteo, c1, setup, oracle_out, ns_t
dev = torch.device('cuda')
for name, mk in [('c1', lambda: c1('head')), ('criteo', lambda: small_criteo('head'))]:
    for B in [64, 128, 129, 200, 512]:
        cfg = mk()
        P, model, batch = setup(cfg, B, dev)
        ns, seq, _ = batch
        with torch.no_grad():
            out = model((ns_t(ns, dev), ns_t(seq, dev)))
        ref = oracle_out(P, cfg, batch)
        lg = model._last_logits[0].double().cpu().numpy()
        e = np.abs(lg - ref['logits']['ctr'].numpy()[:, 0])
        print(name, B, 'max err', e.max(), 'argmax', e.argmax(), 'n bad', (e > 1e-3).sum())
