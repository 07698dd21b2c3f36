"""MI355X-native trust-region inverse-compositional solver for Deep Probabilistic
Feature-metric Tracking (drop-in for the reference's `models.LeastSquareTracking`).

`deep_prob_feature_track_amd.ic` is the torch-facing HIP solver;
`deep_prob_feature_track_amd.models` mirrors the reference's module layout
(`models.LeastSquareTracking`, `models.algorithms`, `models.geometry`).
"""
__version__ = "0.1.0"
