"""Layer implementations; importing this package registers every layer type."""
from . import common, data, loss, neuron, vision  # noqa: F401
