"""Drop-in mirror of the reference's `model` package (AdaptedCLIP, create_model, tokenize)."""
