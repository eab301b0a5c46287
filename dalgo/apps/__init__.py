"""Reference-compatible applications (the bodies of the entry scripts)."""
