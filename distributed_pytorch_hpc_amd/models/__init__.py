"""Model zoo: every architecture the reference trains, defined natively for MI355X."""
from .llama2 import ModelArgs, Transformer, TransformerBlock, build_llama, convert_reference_state_dict, get_preset
from .pp_transformer import PipelineTransformer
from .resnet import ResNet, resnet, resnet18, resnet50, resnet101, resnet152
from .toy import FourBlockMLP, LinearModel, SimpleModel, StageModule, ToyMLP, ToyModel, manual_split_stages
from .unet import SimpleUNet
from .vit import SimpleViT, vit_tp_plan

__all__ = [
    "ModelArgs", "Transformer", "TransformerBlock", "build_llama", "convert_reference_state_dict", "get_preset",
    "PipelineTransformer", "ResNet", "resnet", "resnet18", "resnet50", "resnet101", "resnet152", "FourBlockMLP",
    "LinearModel", "SimpleModel", "StageModule", "ToyMLP", "ToyModel", "manual_split_stages", "SimpleUNet",
    "SimpleViT", "vit_tp_plan",
]
