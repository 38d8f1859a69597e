"""Drop-in for the reference's `simple_knn` extension (scene/gaussian_model.py:20): `_C.distCUDA2`."""
