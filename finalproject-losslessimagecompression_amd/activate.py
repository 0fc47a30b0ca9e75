"""Activation registry (mirror of activate.py:15-17; empty like the reference).
DenseLayer resolves 'ReLU' / 'LeakyReLU' / 'Tanh' itself (nnlayer.py:31-38)."""
import moduleregister


class ActivateFunc(moduleregister.Register):
    def __init__(self):
        super().__init__()
