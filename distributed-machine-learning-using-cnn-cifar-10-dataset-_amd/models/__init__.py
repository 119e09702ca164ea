"""Model families: the reference CIFAR-10 CNN and ResNet-20 (BASELINE config 4)."""
from .cifar_cnn import CifarCNN, PARAM_SPECS, FLAT_SIZE, NUM_PARAMS  # noqa: F401


def build_model(name: str, seed: int = 0, relu_logits: bool = True, flat=None, backend: str = "torch"):
    if name in ("cifar_cnn", "cnn", "cifar10_cnn"):
        return CifarCNN(flat=flat, relu_logits=relu_logits, seed=seed, backend=backend)
    if backend != "torch":
        raise ValueError(f"backend {backend!r} exists for the CIFAR CNN only")
    if name in ("resnet20", "resnet-20"):
        from .resnet import ResNet20
        return ResNet20(flat=flat, seed=seed)   # standard linear logits (the ReLU-logit quirk is the CNN's)
    raise ValueError(f"unknown model {name!r}")
