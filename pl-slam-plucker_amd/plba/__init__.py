"""plba — MI355X-native local bundle adjustment for PL-SLAM (Plücker/orth LBA path)."""
