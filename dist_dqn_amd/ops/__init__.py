"""Device ops: dispatch to the in-tree HIP extension (gfx950) or the torch oracle on CPU."""
