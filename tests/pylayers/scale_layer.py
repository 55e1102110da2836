"""A user Python layer (pycaffe protocol) for tests/test_net.py::test_python_layer."""


class ScaleByParam:
    def setup(self, bottom, top):
        self.k = float(self.param_str or "1.0")

    def reshape(self, bottom, top):
        top[0].reshape(bottom[0].shape, bottom[0].dtype)

    def forward(self, bottom, top):
        top[0].data = bottom[0].data * self.k

    def backward(self, top, propagate_down, bottom):
        if propagate_down[0]:
            bottom[0].diff = top[0].diff * self.k
