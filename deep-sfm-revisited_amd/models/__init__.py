"""Reference-named model modules (models/ of jytime/Deep-SfM-Revisited) for the hot path."""
