"""Model zoo (DSL-built NetParameters + reference solver settings)."""
from .zoo import (MODELS, alexnet, build, caffenet, cifar10_full, cifar10_quick, googlenet, lenet,  # noqa: F401
                  solver_for, vgg16)
