"""spef_amd -- MI355X-native inference target for the Spacecraft Pose Estimation Framework."""
