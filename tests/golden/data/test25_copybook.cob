      ****************************************************************************
      *                                                                          *
      * Copyright 2018 ABSA Group Limited                                        *
      *                                                                          *
      * Licensed under the Apache License, Version 2.0 (the "License");          *
      * you may not use this file except in compliance with the License.         *
      * You may obtain a copy of the License at                                  *
      *                                                                          *
      *     http://www.apache.org/licenses/LICENSE-2.0                           *
      *                                                                          *
      * Unless required by applicable law or agreed to in writing, software      *
      * distributed under the License is distributed on an "AS IS" BASIS,        *
      * WITHOUT WARRANTIES OR CONDITIONS OF ANY KIND, either express or implied. *
      * See the License for the specific language governing permissions and      *
      * limitations under the License.                                           *
      *                                                                          *
      ****************************************************************************

      01 RECORD.
           05  ID                        PIC 9(1).
           05  DATA.
               10  FIELD                 PIC X.
               10  DETAIL1       OCCURS 0 TO 2 TIMES
                                 DEPENDING ON FIELD.
                   15  VAL1       PIC X.
               10  DETAIL2       OCCURS 0 TO 2 TIMES
                                 DEPENDING ON FIELD.
                   15  VAL2       PIC X.
