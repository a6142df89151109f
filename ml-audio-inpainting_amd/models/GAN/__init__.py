"""Drop-in for the reference's models/GAN package (networks, loss, dataset, train)."""
