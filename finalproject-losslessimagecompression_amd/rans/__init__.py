"""Drop-in for the reference's native package `rans` (rans/rans.pyx built by
rans/setup.py): `from rans.rans import encode, decode` works unchanged."""
