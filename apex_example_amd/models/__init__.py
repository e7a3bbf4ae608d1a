"""In-repo model zoo (no torchvision / transformers downloads): the reference
ConvNet, ResNet-18/34/50/101/152, BERT (base/large) and GPT-2 (small/medium)."""
from .convnet import ConvNet  # noqa: F401
from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152  # noqa: F401


def __getattr__(name):
    # transformer models import lazily (they pull in the fused LayerNorm op)
    if name in ("BertConfig", "BertForPreTraining", "bert_large", "bert_base"):
        from . import bert

        return getattr(bert, name)
    if name in ("GPT2Config", "GPT2LMHeadModel", "gpt2_medium", "gpt2_small"):
        from . import gpt2

        return getattr(gpt2, name)
    raise AttributeError(name)
