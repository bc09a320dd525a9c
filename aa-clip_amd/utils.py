"""Drop-in for the reference utils.py entry points used by test.py
(setup_seed :10-20, cos_sim :86-93). Training augmentations are out of scope."""
import os
import random

import numpy as np
import torch


def setup_seed(seed):
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
    random.seed(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    os.environ["PYTHONHASHSEED"] = str(seed)
    # The HIP kernels are deterministic by construction (no atomics, fixed
    # reduction order), so torch's deterministic-algorithms switch is set for
    # parity with the reference but does not gate anything on the path.
    torch.use_deterministic_algorithms(True, warn_only=True)
    os.environ["CUBLAS_WORKSPACE_CONFIG"] = ":4096:8"


def cos_sim(a_norm, b_norm):
    if len(a_norm.shape) == 2:
        return b_norm @ a_norm.transpose(1, 0)
    if len(a_norm.shape) == 1:
        return b_norm @ a_norm
    raise NotImplementedError
