"""Actors: device-resident (batched synthetic envs on the GPU) and Ape-X CPU actor processes."""
