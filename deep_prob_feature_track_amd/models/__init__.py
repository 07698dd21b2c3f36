"""Drop-in mirror of the reference's `models` package (LeastSquareTracking,
algorithms, geometry, submodules) on the HIP U_IC solver."""
