"""clipmi — MI355X-native CLIP dual-encoder + adapter contrastive fine-tuning path.

Drop-in mirrors of the reference's ``model_m.CLIPWithAdapters`` and
``trainer.CLIPAdapterTrainer`` whose compute runs on libclipmi (hand-written HIP for
gfx950, C ABI in include/clipmi.h)."""
from .config import CLIPConfig, PRESETS, TowerConfig, resolve  # noqa: F401


def __getattr__(name):
    # torch-dependent pieces load lazily so config/synth stay importable without a GPU stack
    if name == "CLIPWithAdapters":
        from .model import CLIPWithAdapters
        return CLIPWithAdapters
    if name == "CLIPTokenizer":  # caption BPE of the input step (dataset.py:152-159)
        from .tokenizer import CLIPTokenizer
        return CLIPTokenizer
    if name in ("ContextAdapter", "SharedAdapter", "TextualAdapter"):  # adapter/peclip.py's modules
        from . import peclip
        return getattr(peclip, name)
    if name in ("CLIPAdapterTrainer", "FusedAdamW"):
        from . import trainer
        return getattr(trainer, name)
    raise AttributeError(name)
