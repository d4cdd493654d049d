"""Model families of the reference examples (+ ResNet-50 from BASELINE.json).

* :class:`CifarConvNet` -- examples/cifar10.lua:101-143, examples/Model.lua
* :class:`MnistConvNet` / :class:`MnistMLP` -- examples/mnist.lua:53-66
* :func:`resnet50` -- BASELINE.json config 5 (bucket / xGMI stress)
"""
from .cifar_convnet import CifarConvNet, num_params
from .mnist import MnistConvNet, MnistMLP
from .resnet import ResNet50, resnet50


def make_executor(model, flat, bucketer=None, max_batch=None):
    """Native (hand-written HIP) executor for ``model`` bound to ``flat``."""
    if isinstance(model, CifarConvNet):
        from .cifar_hip import CifarHIPExecutor

        return CifarHIPExecutor(model, flat, bucketer=bucketer, max_batch=max_batch)
    if isinstance(model, MnistConvNet):
        from .mnist_hip import MnistHIPExecutor

        return MnistHIPExecutor(model, flat, bucketer=bucketer, max_batch=max_batch)
    raise NotImplementedError(f"no native executor for {type(model).__name__}")


MODELS = {"cifar10": CifarConvNet, "mnist": MnistConvNet, "mnist_mlp": MnistMLP, "resnet50": ResNet50}


def build_model(name: str, **kw):
    return MODELS[name](**kw)


__all__ = ["CifarConvNet", "MnistConvNet", "MnistMLP", "ResNet50", "resnet50", "num_params", "make_executor",
           "build_model", "MODELS"]
