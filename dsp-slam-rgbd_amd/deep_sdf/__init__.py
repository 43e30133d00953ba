"""DeepSDF decoder loading for the MI355X hot path (replaces the reference's deep_sdf/)."""
