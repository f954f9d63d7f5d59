"""IAP-protected endpoint client: ``python auth.py URL CLIENT_ID [--input FILE]``.

Thin CLI over :mod:`service_account_auth_improvements_amd.utils.iap` (reference: auth.py:98-119).
"""
import sys

from service_account_auth_improvements_amd.utils.iap import main

if __name__ == "__main__":
    sys.exit(main())
