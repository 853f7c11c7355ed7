"""Seeding (torchrec/utils/global_utils.py:7-16)."""
import torch


def set_torch_seed(seed: int) -> None:
    """Seed CPU and every GPU generator; deterministic cuDNN/MIOpen flags."""
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
