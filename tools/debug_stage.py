import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from test_model_gpu import small_criteo, c1, setup, ns_t
from recommend_amd.model import _Tokenize, _Block, _Head
from oracle import onetrans_ref as R
dev = torch.device('cuda')
for name, mk, B in [('c1', lambda: c1('head'), 64), ('criteo', lambda: small_criteo('head'), 64)]:
    cfg = mk()
    P, model, batch = setup(cfg, B, dev)
    ns, seq, _ = batch
    Pt = R.to_torch(P)
    with torch.no_grad():
        for rep in range(2):
            plan = model._plan(ns_t(ns, dev), ns_t(seq, dev))
            x = _Tokenize.apply(model.flat, model, plan)
            xr = R.tokenizer(Pt, cfg, R.to_torch(ns), R.to_torch(seq))
            L0 = xr.shape[1]
            e = (x.double().cpu().view(B, L0, -1) - xr).abs()
            print(name, rep, 'tok err', e.max().item(), 'per-pos max', e.amax((0, 2))[:12].numpy().round(4))
            xg = xr
            sched = cfg.pyramid_schedule(L0)
            for l, s in enumerate(sched):
                Kq = s['keep'] if l < len(sched) - 1 else 1
                # feed the oracle input to isolate the block
                xin = xg.reshape(B * s['in_len'], -1).float().to(dev).contiguous()
                y = _Block.apply(model.flat, xin, model, l, s['in_len'], Kq, 0, False)
                yr = R.block_vectorized(Pt, cfg, l, xg, Kq, False, 0)
                eb = (y.double().cpu().view(B, Kq, -1) - yr).abs()
                print('   block', l, 'I', s['in_len'], 'K', Kq, 'err', eb.max().item())
                xg = yr
