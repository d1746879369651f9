
BPlus214_Output_0J(-╝Gбн⌡6A╢BШаеA┐j┌@ дuа÷╪@Ю÷≤аBэH©А	⌠а