"""Data pipeline: loaders, samplers, host batch sources and the device feeder."""
