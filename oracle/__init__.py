"""Test-infrastructure oracle (CPU restatement of the reference solver). Never imported by the product."""
