"""Stand-in for scikit-image (absent here); only `measure` is referenced by the reference at import."""
