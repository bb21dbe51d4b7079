"""Lead/accompaniment source/filter model (reference: SeparateLeadStereo/)."""
