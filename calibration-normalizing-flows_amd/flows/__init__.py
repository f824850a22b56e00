"""Drop-in mirror of the reference's `flows` package (flows/flows.py, flows/utils.py),
plus the calibrator flow factories the reference's notebooks import
(`flows.realNVP_torch.RealNvpFlow`, `flows.nice_torch.NiceFlow`)."""
