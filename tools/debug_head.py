import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from test_model_gpu import small_criteo, c1, setup, ns_t, oracle_out
from recommend_amd.model import _Tokenize, _Block, _Head
from oracle import onetrans_ref as R
dev = torch.device('cuda')
cfg = c1('head'); B = 64
P, model, batch = setup(cfg, B, dev)
ns, seq, lab = batch
Pt = R.to_torch(P)
ref = oracle_out(P, cfg, batch)
with torch.no_grad():
    for rep in range(3):
        out = model((ns_t(ns, dev), ns_t(seq, dev)), training=False)
        lg = model._last_logits[0].double().cpu().numpy()
        print('full', rep, np.abs(lg - ref['logits']['ctr'].numpy()[:, 0]).max())
    # head on oracle input
    xr = R.tokenizer(Pt, cfg, R.to_torch(ns), R.to_torch(seq))
    for l, s in enumerate(cfg.pyramid_schedule(xr.shape[1])):
        xr = R.block_vectorized(Pt, cfg, l, xr, 1 if l == cfg.num_layers - 1 else s['keep'], False, 0)
    xl = xr[:, -1].float().to(dev).contiguous()
    probs = _Head.apply(model.flat, xl, model)
    print('head only', np.abs(model._last_logits[0].double().cpu().numpy() - ref['logits']['ctr'].numpy()[:, 0]).max())
    print('probs vs logits', probs[0, :4].cpu().numpy(), ref['probs']['ctr'][:4, 0].numpy())
    print('out dict', out['ctr'][:4, 0].cpu().numpy())
