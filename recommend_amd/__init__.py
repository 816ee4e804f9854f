"""recommend_amd — MI355X-native OneTrans ranking path (training step fwd+bwd) behind the reference's
package API (``rank/scaling_up/oneTrans/practice/__init__.py:9-26``).

The arithmetic runs in ``libonetrans_hip.so`` (gfx950 HIP kernels, C ABI in
``include/onetrans_hip.h``).  Importing this package does not need a GPU; constructing a model does.
"""

__version__ = '1.0.0'

from .config import OneTransConfig, get_model_config, workload_config  # noqa: F401
from .data import create_sample_batch, criteo_batch, make_batch  # noqa: F401
from .features import DataLoader, FeatureProcessor, OneTransDataset, SequenceProcessor  # noqa: F401
from .metrics import auc, keras_auc  # noqa: F401


def __getattr__(name):
    # model / trainer pull in torch + the HIP library lazily
    if name in ('OneTransModel', 'create_onetrans_model'):
        from . import model
        return getattr(model, name)
    if name in ('OneTransTrainer', 'train_one_trans_model', 'OneTransOptimizer'):
        from . import trainer
        return getattr(trainer, name)
    raise AttributeError(name)


__all__ = ['OneTransModel', 'OneTransConfig', 'get_model_config', 'DataLoader', 'FeatureProcessor',
           'SequenceProcessor', 'OneTransDataset', 'OneTransTrainer', 'train_one_trans_model', 'create_sample_batch', 'criteo_batch', 'make_batch', 'workload_config', 'auc', 'keras_auc']
